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
