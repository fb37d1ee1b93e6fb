"""C-ABI checks that need no GPU: the library loads, exports exactly what include/hipquorum.h
declares, the ctypes struct mirrors match the C layout, and argument validation fails cleanly."""
import ctypes
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "hipquorum.h")


def declared_functions():
    text = open(HEADER).read()
    return sorted(set(re.findall(r"^(?:int|void|const char \*)\s*\*?(hq_\w+)\(", text, re.M)))


def test_exports_match_header(hq):
    names = declared_functions()
    assert len(names) >= 20
    out = subprocess.run(["nm", "-D", "--defined-only", hq.LIB_PATH], capture_output=True,
                         text=True, check=True).stdout
    exported = sorted(set(re.findall(r" T (hq_\w+)$", out, re.M)))
    assert exported == names
    assert sorted(hq.SIGNATURES) == names   # the binding declares every entry point
    for n in names:
        assert getattr(hq.lib, n)


def test_abi_version(hq):
    assert hq.lib.hq_abi_version() == hq.HQ_ABI_VERSION == 21


LAYOUT_C = r"""
#include <stdio.h>
#include <stddef.h>
#include "hipquorum.h"
#define F(T, m) printf(#T "." #m " %zu\n", offsetof(T, m));
int main(void) {
  printf("hq_commit_args %zu\n", sizeof(hq_commit_args));
  printf("hq_synth_spec %zu\n", sizeof(hq_synth_spec));
  F(hq_commit_args, G) F(hq_commit_args, n_max) F(hq_commit_args, form)
  F(hq_commit_args, ring_len) F(hq_commit_args, match_stride) F(hq_commit_args, match)
  F(hq_commit_args, n_voting) F(hq_commit_args, committed_in) F(hq_commit_args, committed_out)
  F(hq_commit_args, last_index) F(hq_commit_args, term_start) F(hq_commit_args, term)
  F(hq_commit_args, ring) F(hq_commit_args, changed) F(hq_commit_args, fallback)
  F(hq_commit_args, term_mask) F(hq_commit_args, ring32) F(hq_commit_args, layout)
  for (unsigned n = 1; n <= 8; ++n)
    for (unsigned f = 0; f <= 3; ++f)
      printf("tile_words_%u_%u %llu\nlead_words_%u_%u %llu\n", n, f,
             (unsigned long long)hq_commit_tile_words(n, f), n, f,
             (unsigned long long)hq_commit_tile_words_for(n, f, HQ_LAYOUT_TILES_LEADER));
  printf("tiles_129 %llu\n", (unsigned long long)hq_commit_tiles(129));
  printf("hq_commit_lag_args %zu\n", sizeof(hq_commit_lag_args));
  F(hq_commit_lag_args, G) F(hq_commit_lag_args, n_max) F(hq_commit_lag_args, form)
  F(hq_commit_lag_args, ring_len) F(hq_commit_lag_args, flags)
  F(hq_commit_lag_args, lag_stride) F(hq_commit_lag_args, lag)
  printf("lag_leader_flag %u\nlayout_leader %u\n", (unsigned)HQ_LAG_LEADER_IMPLICIT,
         (unsigned)HQ_LAYOUT_TILES_LEADER);
  F(hq_commit_lag_args, n_voting) F(hq_commit_lag_args, cin_lag) F(hq_commit_lag_args, cout_lag)
  F(hq_commit_lag_args, ts_lag) F(hq_commit_lag_args, lag_mask) F(hq_commit_lag_args, changed)
  F(hq_commit_lag_args, fallback)
  F(hq_synth_spec, seed) F(hq_synth_spec, G) F(hq_synth_spec, cid_base)
  F(hq_synth_spec, cid_stride) F(hq_synth_spec, n_max) F(hq_synth_spec, mixed_n)
  F(hq_synth_spec, ring_len) F(hq_synth_spec, parity_extras)
  printf("hq_member %zu\n", sizeof(hq_member));
  printf("hq_group_view %zu\n", sizeof(hq_group_view));
  printf("hq_msg %zu\n", sizeof(hq_msg));
  printf("hq_match_update %zu\n", sizeof(hq_match_update));
  printf("hq_append_update %zu\n", sizeof(hq_append_update));
  F(hq_member, node_id) F(hq_member, match) F(hq_member, role) F(hq_member, active)
  F(hq_group_view, node_id) F(hq_group_view, committed) F(hq_group_view, last_index)
  F(hq_group_view, term_start) F(hq_group_view, term) F(hq_group_view, ctx_low)
  F(hq_group_view, ctx_high) F(hq_group_view, term_mask) F(hq_group_view, first_member)
  F(hq_group_view, n_members) F(hq_group_view, first_msg) F(hq_group_view, n_msgs)
  F(hq_msg, from) F(hq_msg, hint_low) F(hq_msg, hint_high) F(hq_msg, reject)
  printf("hq_wire_message %zu\n", sizeof(hq_wire_message));
  F(hq_wire_message, ev) F(hq_wire_message, cluster_id) F(hq_wire_message, to)
  F(hq_wire_message, log_term) F(hq_wire_message, commit) F(hq_wire_message, n_entries)
  F(hq_wire_message, has_snapshot)
  printf("hq_wire_batch_info %zu\nhq_wire_stats %zu\nbin_ver %u\n", sizeof(hq_wire_batch_info),
         sizeof(hq_wire_stats), (unsigned)HQ_RPC_BIN_VERSION);
  printf("in_place %u\ngrouped %u\n", (unsigned)HQ_LAYOUT_IN_PLACE, (unsigned)HQ_INGEST_GROUPED);
  printf("hq_engine_config %zu\nhq_engine_stats %zu\nengine_signal %u\n",
         sizeof(hq_engine_config), sizeof(hq_engine_stats), (unsigned)HQ_ENGINE_SIGNAL);
  F(hq_engine_config, n_max) F(hq_engine_config, form) F(hq_engine_config, layout)
  F(hq_engine_config, ring_len) F(hq_engine_config, depth) F(hq_engine_config, flags)
  F(hq_engine_config, idle_us) F(hq_engine_config, max_workgroups)
  F(hq_engine_stats, posted) F(hq_engine_stats, completed) F(hq_engine_stats, relaunches)
  F(hq_engine_stats, grid) F(hq_engine_stats, block) F(hq_engine_stats, depth)
  F(hq_engine_stats, running)
  printf("hq_event16 %zu\nhq_event %zu\nev16_flags %u\n", sizeof(hq_event16), sizeof(hq_event),
         (unsigned)(HQ_EV16_READ_CTX | HQ_EV16_FULL << 8));
  F(hq_event16, kind) F(hq_event16, type) F(hq_event16, from) F(hq_event16, term)
  F(hq_event16, value)
  printf("hq_step_output %zu\nhq_step_stream %zu\nhq_encode16_job %zu\n", sizeof(hq_step_output),
         sizeof(hq_step_stream), sizeof(hq_encode16_job));
  F(hq_step_output, ready_compact) F(hq_step_output, gpu_ns) F(hq_step_output, gpu_jobs)
  F(hq_step_output, wait_sleeps) F(hq_step_output, wait_end_ns) F(hq_step_output, device_end_ticks)
  F(hq_step_output, ready_slots) F(hq_step_output, n_ready_slotted)
  F(hq_step_output, device_start_ticks)
  F(hq_step_stream, sizes16) F(hq_encode16_job, sizes16)
  printf("wait_modes %u,%u,%u,%u,%u\nready_slots_flag %u\n", (unsigned)HQ_WAIT_BLOCK,
         (unsigned)HQ_WAIT_SLEEP, (unsigned)HQ_WAIT_SPIN, (unsigned)HQ_WAIT_CLOCK,
         (unsigned)HQ_WAIT_ADAPT,
         (unsigned)HQ_WORKER_READY_SLOTS);
  return 0;
}
"""


def test_struct_layout_matches_c(hq, tmp_path):
    src = tmp_path / "layout.c"
    src.write_text(LAYOUT_C)
    exe = tmp_path / "layout"
    subprocess.run(["gcc", "-std=c11", "-I", os.path.join(ROOT, "include"), "-o", str(exe),
                    str(src)], check=True)
    lines = subprocess.run([str(exe)], capture_output=True, text=True, check=True).stdout.split("\n")
    c = dict(l.rsplit(" ", 1) for l in lines if l)
    assert int(c["hq_commit_args"]) == ctypes.sizeof(hq.CommitArgs)
    assert int(c["hq_synth_spec"]) == ctypes.sizeof(hq.SynthSpec)
    assert int(c["hq_commit_lag_args"]) == ctypes.sizeof(hq.LagArgs)
    assert int(c["hq_engine_config"]) == ctypes.sizeof(hq.EngineConfig)
    assert int(c["hq_engine_stats"]) == ctypes.sizeof(hq.EngineStats)
    assert int(c["engine_signal"]) == hq.HQ_ENGINE_SIGNAL
    dtypes = {"hq_member": hq.MEMBER_DTYPE, "hq_group_view": hq.GROUP_DTYPE,
              "hq_msg": hq.MSG_DTYPE, "hq_wire_message": hq.WIRE_MESSAGE_DTYPE,
              "hq_event16": hq.EVENT16_DTYPE, "hq_event": hq.EVENT_DTYPE}
    assert int(c["ev16_flags"]) == hq.EV16_READ_CTX | hq.EV16_FULL << 8
    assert int(c["hq_wire_batch_info"]) == ctypes.sizeof(hq.WireBatchInfo)
    assert int(c["hq_wire_stats"]) == ctypes.sizeof(hq.WireStats)
    assert int(c["bin_ver"]) == hq.HQ_RPC_BIN_VERSION
    assert int(c["in_place"]) == hq.HQ_LAYOUT_IN_PLACE
    # the step worker's structs (ABI 21: wait clocks, ReadyToRead slots, 2-byte size words)
    for t, py in (("hq_step_output", hq.StepOutput), ("hq_step_stream", hq.StepStream),
                  ("hq_encode16_job", hq.Encode16Job)):
        assert int(c[t]) == ctypes.sizeof(py), t
        for f in [k for k in c if k.startswith(t + ".")]:
            assert int(c[f]) == getattr(py, f.split(".", 1)[1]).offset, f
    assert c["wait_modes"] == ",".join(map(str, (hq.HQ_WAIT_BLOCK, hq.HQ_WAIT_SLEEP, hq.HQ_WAIT_SPIN,
                                                 hq.HQ_WAIT_CLOCK, hq.HQ_WAIT_ADAPT)))
    assert int(c["ready_slots_flag"]) == hq.HQ_WORKER_READY_SLOTS
    assert int(c["grouped"]) == hq.HQ_INGEST_GROUPED
    for name, dt in dtypes.items():
        assert int(c[name]) == dt.itemsize, name
    assert int(c["hq_match_update"]) == 16 and int(c["hq_append_update"]) == 16
    for n in range(1, 9):
        for f in range(4):
            assert int(c[f"tile_words_{n}_{f}"]) == hq.commit_tile_words(n, f)
            assert int(c[f"lead_words_{n}_{f}"]) == hq.commit_tile_words(
                n, f, hq.HQ_LAYOUT_TILES_LEADER)
    assert int(c["lag_leader_flag"]) == hq.HQ_LAG_LEADER_IMPLICIT
    assert int(c["layout_leader"]) == hq.HQ_LAYOUT_TILES_LEADER
    assert int(c["tiles_129"]) == hq.commit_tiles(129) == 2
    for key, val in c.items():
        if "." in key:
            t, m = key.split(".")
            if t in dtypes:
                assert dtypes[t].fields[m][1] == int(val), key
                continue
            cls = {"hq_commit_args": hq.CommitArgs, "hq_synth_spec": hq.SynthSpec,
                   "hq_commit_lag_args": hq.LagArgs, "hq_engine_config": hq.EngineConfig,
                   "hq_engine_stats": hq.EngineStats, "hq_step_output": hq.StepOutput,
                   "hq_step_stream": hq.StepStream, "hq_encode16_job": hq.Encode16Job}[t]
            assert getattr(cls, m).offset == int(val), key


def test_null_context_is_invalid(hq):
    a = hq.CommitArgs()
    assert hq.lib.hq_commit_dev(None, ctypes.byref(a)) == hq.HQ_E_INVAL
    assert hq.lib.hq_sync(None) == hq.HQ_E_INVAL
    assert hq.lib.hq_readindex_dev(None, 0, None, None, 3, None, None) == hq.HQ_E_INVAL
    assert hq.lib.hq_vote_dev(None, 0, None, None, None, 3, None, None) == hq.HQ_E_INVAL
    assert hq.lib.hq_commit_lag_dev(None, ctypes.byref(hq.LagArgs())) == hq.HQ_E_INVAL
    assert hq.lib.hq_commit_fused_dev(None, None, 0) == hq.HQ_E_INVAL
    assert hq.lib.hq_commit_lag_fused_dev(None, None, 0) == hq.HQ_E_INVAL
    assert hq.lib.hq_wait_for(None, None) == hq.HQ_E_INVAL
    hq.lib.hq_close(None)  # no-op
    assert hq.lib.hq_engine_open(None, None, None) == hq.HQ_E_INVAL
    assert hq.lib.hq_engine_post(None, None, 0, None) == hq.HQ_E_INVAL
    assert hq.lib.hq_engine_wait(None, 0) == hq.HQ_E_INVAL
    assert hq.lib.hq_engine_drain(None) == hq.HQ_E_INVAL
    hq.lib.hq_engine_close(None)  # no-op
    assert hq.lib.hq_last_error(None) is not None


def test_open_without_gpu_fails_cleanly(hq):
    if hq.device_count() > 0:
        pytest.skip("a GPU is visible: covered by the gpu tests")
    with pytest.raises(hq.HQError) as e:
        hq.Context(0)
    assert e.value.code == hq.HQ_E_DEVICE
    assert "no HIP device" in str(e.value)


def test_kernels_are_gfx950(hq):
    """The fat binary carries gfx950 code objects only (no other offload target)."""
    blob = open(hq.LIB_PATH, "rb").read()
    targets = set(re.findall(rb"amdgcn-amd-amdhsa-+(gfx[0-9a-z]+)", blob))
    assert targets == {b"gfx950"}, targets


def test_worker_without_gpu_fails_cleanly(hq):
    if hq.device_count() > 0:
        pytest.skip("a GPU is visible: covered by tests/test_gpu_worker.py")
    with pytest.raises(hq.HQError) as e:
        hq.Worker(0, 5)
    assert e.value.code == hq.HQ_E_DEVICE
    assert hq.lib.hq_worker_open(0, 0, ctypes.byref(ctypes.c_void_p())) == hq.HQ_E_INVAL
    assert hq.lib.hq_worker_step(None, None, None) == hq.HQ_E_INVAL
    hq.lib.hq_worker_close(None)   # no-op
