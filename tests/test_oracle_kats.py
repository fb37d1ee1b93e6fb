"""The CPU oracle against the reference's own known-answer tables (tests/golden/).

These pin oracle/qref.c before it is trusted as the parity checker for the HIP kernels.
"""

import numpy as np
import pytest

from oracle import qref

from kats import COMMIT_TABLES, KATS



def _log(case, committed=None):
    terms = {int(k): v for k, v in case["log"].items()}
    c = case.get("committed", 0) if committed is None else committed
    return qref.EntryLog(case["first_minus_1"], case["last"], c, terms)


@pytest.mark.parametrize("table", COMMIT_TABLES)
def test_commit_tables(table):
    for case in KATS[table]:
        log = _log(case)
        rc, q = qref.try_commit(case["remotes"], case["witnesses"], log, case["term"])
        assert rc in (0, 1), case
        assert log.committed == case["want_committed"], (table, case)
        # independent count-based definition of the quorum match
        m = np.array(case["remotes"] + case["witnesses"], np.uint64)
        assert q == int(qref.lib.qref_quorum_match_by_count(m.ctypes.data, len(m)))


def test_sort_match_values():
    for case in KATS["TestUnrolledBubbleSortMatchValue"]:
        assert qref.sort_match_values(case["vals"]) == case["want"]


def test_quorum_values():
    for case in KATS["TestQuorumValue"]:
        assert qref.quorum(case["n"]) == case["quorum"]
    for case in KATS["TestIsSingleNodeQuorum"]:
        assert bool(qref.lib.qref_is_single_node_quorum(case["n"])) == case["single"]


@pytest.mark.parametrize("table", ["TestTerm", "TestTermWithUnstableSnapshot", "TestInMemGetTerm",
                                   "TestInMemGetTermReturnSnapshotTerm"])
def test_term_tables(table):
    for case in KATS[table]:
        assert _log(case, 0).term(case["index"]) == case["want"], case


@pytest.mark.parametrize("table", ["TestReadIndexLeaderCanBeConfirmed",
                                   "TestSameCtxCanNotBeAddedTwice",
                                   "TestReadIndexRequestCanBeAdded",
                                   "TestReadIndexChecksInputIndex"])
def test_readindex_tables(table):
    t = KATS[table]
    ri = qref.PyReadIndex()
    for op in t["ops"]:
        if op[0] == "add":
            assert ri.add_request(op[1], tuple(op[2]), op[3]) == 0
        elif op[0] == "add_panics":
            assert ri.add_request(op[1], tuple(op[2]), op[3]) == qref.QREF_PANIC
        else:
            got = ri.confirm(tuple(op[1]), op[2], op[3])
            want = op[4]
            if want is None:
                assert got is None
            else:
                assert got == [(w[0], w[1], tuple(w[2])) for w in want]
    if "final_pending" in t:
        assert ri.n_pending == t["final_pending"]
        assert ri.n_queue == t["final_queue"]


def test_handle_vote_resp():
    v = qref.PyVotes()
    for frm, rej, want in KATS["TestHandleVoteResp"]["seq"]:
        assert v.handle_vote_resp(frm, rej) == want


def test_leader_election_in_one_round():
    for case in KATS["TestLeaderElectionInOneRoundRPC"]:
        n = case["size"]
        q = qref.quorum(n)
        v = qref.PyVotes()
        # campaign: self vote then single-node short-cut (raft.go:1093-1097)
        v.handle_vote_resp(1, False)
        state = qref.QREF_LEADER if q == 1 else qref.QREF_CANDIDATE
        for frm, granted in case["votes"].items():
            if state != qref.QREF_CANDIDATE:
                break
            state = v.candidate_resp(int(frm), not granted, False, q)
        assert state == case["want_state"], case
        # the bitmap form the kernel consumes gives the same outcome
        g = np.array([1 | sum(1 << (int(k) - 1) for k, x in case["votes"].items() if x)], np.uint8)
        r = np.array([sum(1 << (int(k) - 1) for k, x in case["votes"].items() if not x)], np.uint8)
        out, _ = qref.vote_batch(g, r, None, n)
        assert int(out[0]) & 3 == case["want_state"]


def test_candidate_request_vote_resp():
    for case in KATS["TestHandleCandidateRequestVoteResp"]:
        v = qref.PyVotes()
        q = qref.quorum(case["n"])
        state = qref.QREF_CANDIDATE
        for frm, rej in case["msgs"]:
            state = v.candidate_resp(frm, rej, False, q)
            if state != qref.QREF_CANDIDATE:
                break
        assert state == case["want_state"]


def test_observer_vote_dropped():
    v = qref.PyVotes()
    assert v.candidate_resp(9, False, True, 1) == qref.QREF_CANDIDATE
    assert v.c.n == 0


def test_leader_has_quorum():
    for case in KATS["TestLeaderHasQuorum"]:
        n = case["n"]
        ids = np.arange(1, n + 1, dtype=np.uint64)
        act = np.array(case["active"], np.int32)
        got = qref.lib.qref_leader_has_quorum(ids.ctypes.data, act.ctypes.data, n, 1)
        assert bool(got) == case["want"]
        assert not act.any()  # every active flag reset (remote.go:196-198)
        a = np.array([sum(1 << i for i, x in enumerate(case["active"]) if x)], np.uint8)
        hq, fb, a2 = qref.check_quorum_batch(a, None, n, 0)
        assert bool(hq[0] & 1) == case["want"] and a2[0] == 0 and fb[0] == 0


def test_readindex_single_ctx_quorum():
    # readindex.go:84 — len(confirmed) + 1 >= quorum, distinct senders only
    for n in range(1, 9):
        q = qref.quorum(n)
        for acks in range(0, n):
            ri = qref.PyReadIndex()
            ri.add_request(0, (1, 1), 1)
            got = None
            for frm in range(2, 2 + acks):
                got = ri.confirm((1, 1), frm, q) or got
                ri.confirm((1, 1), frm, q)  # duplicate ack never double counts
            assert (got is not None) == (acks + 1 >= q and acks > 0)


def test_commit_count_definition_random():
    rng = np.random.default_rng(7)
    for _ in range(3000):
        n = int(rng.integers(1, 9))
        m = rng.integers(0, 6, n).astype(np.uint64)
        s = np.sort(m)
        q = s[n - qref.quorum(n)]
        assert q == qref.lib.qref_quorum_match_by_count(m.ctypes.data, n)
        assert qref.sort_match_values(list(m)) == [int(x) for x in s]
