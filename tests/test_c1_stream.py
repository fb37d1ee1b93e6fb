"""BASELINE config C1 — the reference's CPU case: one raft group x 3 voters, tryCommit once per
ReplicateResp on a synthetic match stream (raft.go:1671-1700, :888-909).

The batching claim of DESIGN.md §1 made concrete: deciding every step of the stream as an
independent group against the initial committed index, then taking a running maximum, gives
exactly the committed index the sequential per-message tryCommit produces after every step.
CPU: the oracle's batch form against its sequential replay. GPU: the commit kernel over the
whole stream in one launch, prefix max on the host, against the sequential replay."""
import numpy as np
import pytest

from oracle import qref

T, C0, L0, TS = 200_000, 1000, 1005, 1003   # term_start: the leader's no-op index


def stream(seed=0x5EED0000):
    match, last = qref.c1_stream(seed, T, C0, L0)
    return match, last, qref.c1_run(match, last, TS, C0)


def test_c1_stream_advances_and_is_monotone():
    match, last, seq = stream()
    assert seq[-1] > C0 + T // 16
    assert (np.diff(seq.astype(np.int64)) >= 0).all()
    assert (seq <= last).all()


def test_batched_stream_equals_sequential_on_cpu():
    match, last, seq = stream()
    out = np.zeros(T, np.uint64)
    c0 = np.full(T, C0, np.uint64)
    ts = np.full(T, TS, np.uint64)
    a = qref.commit_args(T, 3, 0, 16, match, c0, out, last, term_start=ts)
    assert qref.commit_batch(a, 4) == 0
    np.testing.assert_array_equal(np.maximum.accumulate(out), seq)


@pytest.mark.gpu
def test_batched_stream_on_gpu_equals_sequential(gpu_ctx, hq):
    match, last, seq = stream(0x5EED0007)
    d = {k: gpu_ctx.upload(v) for k, v in dict(
        match=match, c0=np.full(T, C0, np.uint64), last=last,
        ts=np.full(T, TS, np.uint64)).items()}
    out = gpu_ctx.empty(T, np.uint64)
    a = hq.CommitArgs()
    a.G, a.n_max, a.form, a.ring_len, a.match_stride = T, 3, hq.HQ_FORM_TERM_START, 16, T
    a.match, a.committed_in, a.committed_out = d["match"].ptr, d["c0"].ptr, out.ptr
    a.last_index, a.term_start = d["last"].ptr, d["ts"].ptr
    gpu_ctx.commit_dev(a)
    np.testing.assert_array_equal(np.maximum.accumulate(gpu_ctx.download(out)), seq)
    for x in list(d.values()) + [out]:
        gpu_ctx.free(x)
