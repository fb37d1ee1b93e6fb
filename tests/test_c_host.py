"""The C-ABI from plain C hosts (examples/, no Python or torch in the process): they compile as
C99 against include/hipquorum.h and link libhipquorum.so on the CPU; on the GPU commit_kats.c
decides the reference's TestCommit table (raft_etcd_test.go:1111-1160) in one hq_commit call and
step_worker.c steps three groups (a witness-carried commit, a ReadIndex release, an election)
through a device worker fed a sized event stream."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIBDIR = os.path.join(ROOT, "dragonboat_amd", "lib")


def build(tmp_path, name="commit_kats"):
    exe = str(tmp_path / name)
    subprocess.run(["gcc", "-std=c99", "-Wall", "-Wextra", "-Werror",
                    "-I", os.path.join(ROOT, "include"), os.path.join(ROOT, "examples",
                                                                       name + ".c"),
                    "-L", LIBDIR, "-lhipquorum", f"-Wl,-rpath,{LIBDIR}", "-o", exe], check=True)
    return exe


@pytest.mark.parametrize("name", ["commit_kats", "step_worker"])
def test_c_host_builds(tmp_path, name):
    assert os.path.exists(build(tmp_path, name))


@pytest.mark.gpu
def test_c_host_decides_test_commit(tmp_path):
    r = subprocess.run([build(tmp_path)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert r.stdout.count(" ok") == 14


@pytest.mark.gpu
def test_c_host_steps_a_device_worker(tmp_path):
    r = subprocess.run([build(tmp_path, "step_worker")], capture_output=True, text=True,
                       timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert r.stdout.count(" ok") == 7 and "FAILED" not in r.stdout
