"""The step oracle (oracle/qref_step.c) against the reference's own raft-level tests, restated
as step scenarios in tests/step_scenarios.py (file:line on each). This pins the sequential
checker the GPU step worker is compared with (tests/test_gpu_worker.py)."""
import pytest

import step_scenarios as sc
from step_harness import OracleBackend

CASES = list(sc.all_cases())


def test_scenarios_cover_the_reference_tables():
    names = {c["name"].rstrip("0123456789") for c in CASES}
    assert {"election", "candvote", "checkq", "commit", "ri_single", "ri_unknown", "ri_queue",
            "ri_witness", "ri_observer", "ri_prefix", "single_commit"} <= names
    assert sum(c["name"].startswith("commit") for c in CASES) >= 20
    assert sum(c["name"].startswith("election") for c in CASES) == 13


@pytest.mark.parametrize("case", CASES, ids=[c["name"] for c in CASES])
def test_oracle_scenario(case):
    outs, state = sc.run_case(OracleBackend(), case)
    sc.check_case(case, outs, state)


def test_campaign_state_changes():
    """campaign: becomeCandidate at term+1 (raft.go:959-975), then the vote outcome; a single
    node becomes leader at once and commits its no-op (raft.go:1093-1097, 911-922)."""
    b = OracleBackend()
    b.add_group(1, 1, 4, sc.FOLLOWER, 9, 9, 9, sc.members(1))
    out = b.step({1: [("campaign",)]})[1]
    assert out["states"] == [(5, sc.CANDIDATE, sc.R_CAMPAIGN), (5, sc.LEADER, sc.R_VOTE)]
    assert out["committed"] == 10 and b.state(1)[3:5] == (10, 10)


def test_higher_term_message_steps_down():
    """onMessageTermNotMatched (raft.go:1416-1452): a higher-term response makes the leader a
    follower; the response itself then has no handler."""
    b = OracleBackend()
    b.add_group(1, 1, 3, sc.LEADER, 5, 6, 5, [(1, 6, 0, 0), (2, 5, 0, 0), (3, 5, 0, 0)])
    out = b.step({1: [sc.msg(sc.RREP, 2, 3, 6), sc.msg(sc.RREP, 3, 4, 6),
                      sc.msg(sc.RREP, 2, 4, 6)]})[1]
    assert out["committed"] == 6       # the first message committed 6 at term 3
    assert out["states"] == [(4, sc.FOLLOWER, sc.R_HIGHER)]
    term, st, committed, last, ts, mem, reads = b.state(1)
    assert (term, st) == (4, sc.FOLLOWER)
    assert [m[1] for m in mem] == [6, 0, 0]   # reset(): remotes' match cleared


def test_follower_forwards_reads_and_proposals():
    b = OracleBackend()
    b.add_group(1, 1, 3, sc.FOLLOWER, 5, 6, 5, sc.members(3))
    out = b.step({1: [("read", 1, 2), sc.msg(sc.READIDX, 2, 3, hint=4), ("propose", 2)]})[1]
    assert out["deferred"] == [0, 1, 2]


@pytest.mark.parametrize("idx,want", [(1, 0), (2, 0), (3, 3)])
def test_leader_only_commits_log_from_current_term_with_a_real_log(idx, want):
    """TestLeaderOnlyCommitsLogFromCurrentTerm (raft_etcd_paper_test.go:854-885) over the log the
    reference test builds, held as a term history: entries {1: t1, 2: t2}, the node at term 2
    campaigns (term 3), wins its vote, appends the no-op at 3 (term 3) and a proposal at 4; a
    ReplicateResp from node 2 at `idx` commits only an index of term 3."""
    b = OracleBackend()
    b.add_group(1, 1, 2, sc.FOLLOWER, 0, 2, 2, sc.members(3), log=(0, [(0, 0), (1, 1), (2, 2)]))
    out = b.step({1: [sc.msg(sc.VRESP, 2, 0), ("campaign",)]})[1]
    assert out["states"][-1][:2] == (3, sc.CANDIDATE)
    out = b.step({1: [sc.msg(sc.VRESP, 2, 3), ("propose", 1)]})[1]
    assert out["states"] == [(3, sc.LEADER, sc.R_VOTE)]
    assert b.groups[1].log_terms() == (0, [(0, 0), (1, 1), (2, 2), (3, 3)])
    out = b.step({1: [sc.msg(sc.RREP, 2, 3, idx)]})[1]
    assert out["committed"] == want


def test_term_check_reads_the_history_not_term_start():
    """A leader at term 7 whose log holds terms 2, 4, 6 below its first term-7 entry (90): a
    quorum at 85 (term 6) does not commit, at 95 it does; a ReadIndex needs a committed entry
    at term 7 (raft.go:1612-1621), so it is dropped until the commit. Compacted indexes
    (below first - 1 = 30) have term 0 (logentry.go:143-160)."""
    b = OracleBackend()
    hist = (30, [(0, 2), (40, 4), (70, 6), (90, 7)])
    b.add_group(1, 1, 7, sc.LEADER, 80, 100, 90,
                [(1, 100, 0, 0), (2, 80, 0, 0), (3, 80, 0, 0)], log=hist)
    out = b.step({1: [("read", 11, 1), sc.msg(sc.RREP, 2, 7, 85)]})[1]
    assert out["dropped"] == [(11, 1, 0, sc.D_NOT_READY)] and out["committed"] == 80
    out = b.step({1: [sc.msg(sc.RREP, 3, 7, 95)]})[1]
    assert out["committed"] == 95
    out = b.step({1: [("read", 12, 1)]})[1]
    assert out["dropped"] == [] and b.state(1)[6][0][0] == 95   # pending at index 95
    # a history whose runs are not increasing, or compacted above committed, is refused
    with pytest.raises(AssertionError):
        OracleBackend().add_group(2, 1, 7, sc.LEADER, 80, 100, 90, sc.members(3),
                                  log=(30, [(0, 4), (40, 2)]))
    with pytest.raises(AssertionError):
        OracleBackend().add_group(2, 1, 7, sc.LEADER, 80, 100, 90, sc.members(3),
                                  log=(81, [(0, 4)]))


def test_random_histories_are_valid_and_consistent_with_term_start():
    """The differential tests' histories (tests/step_random.py): every leader's last run starts
    at its term_start at its term, every earlier run is older — the invariant under which the
    worker's term_start <= q <= last check is the history's term(q) == term."""
    import numpy as np

    import step_random as sr
    from oracle import qref

    rng = np.random.default_rng(7)
    multi = 0
    for g in sr.random_groups(rng, 4000):
        qref.StepGroup(*g)                       # accepted by qref_group_set_log
        fm, runs = g[8]
        assert fm <= g[4] and runs[0][0] == 0
        if g[3] == sc.LEADER:
            assert runs[-1] == (g[6], g[2]) and all(t < g[2] for _, t in runs[:-1])
            multi += len(runs) > 2
    assert multi > 500
