"""The C-ABI from a plain C host (examples/commit_kats.c, no Python or torch in the process):
it compiles as C99 against include/hipquorum.h and links libhipquorum.so on the CPU; on the GPU it
decides the reference's TestCommit table (raft_etcd_test.go:1111-1160) in one hq_commit call."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIBDIR = os.path.join(ROOT, "dragonboat_amd", "lib")


def build(tmp_path):
    exe = str(tmp_path / "commit_kats")
    subprocess.run(["gcc", "-std=c99", "-Wall", "-Wextra", "-Werror",
                    "-I", os.path.join(ROOT, "include"), os.path.join(ROOT, "examples",
                                                                       "commit_kats.c"),
                    "-L", LIBDIR, "-lhipquorum", f"-Wl,-rpath,{LIBDIR}", "-o", exe], check=True)
    return exe


def test_c_host_builds(tmp_path):
    assert os.path.exists(build(tmp_path))


@pytest.mark.gpu
def test_c_host_decides_test_commit(tmp_path):
    r = subprocess.run([build(tmp_path)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert r.stdout.count(" ok") == 14
