"""Step-level scenarios restating the reference's own raft tests (file:line on each). Every
scenario runs on any backend of tests/step_harness.py: the CPU oracle (test_oracle_step.py pins
it against these) and the GPU step worker (test_gpu_worker.py)."""
from kats import COMMIT_TABLES, KATS
from oracle.qref import QREF_CANDIDATE as CANDIDATE
from oracle.qref import QREF_FOLLOWER as FOLLOWER
from oracle.qref import QREF_LEADER as LEADER

REMOTE, OBSERVER, WITNESS = 0, 1, 2
RREP, VRESP, HBRESP, READIDX = 13, 15, 18, 19
R_VOTE, R_CQ, R_HIGHER, R_CAMPAIGN = 1, 2, 3, 4
D_WITNESS, D_NOT_READY = 1, 2


def msg(t, frm, term=0, index=0, hint=0, high=0, reject=0):
    return ("msg", t, frm, term, index, hint, high, reject)


def members(n, active=None, witnesses=(), observers=()):
    m = [(i, 0, REMOTE, int(active[i - 1]) if active else 0) for i in range(1, n + 1)]
    m += [(w, 0, WITNESS, 0) for w in witnesses]
    m += [(o, 0, OBSERVER, 0) for o in observers]
    return m


def election_cases():
    """TestLeaderElectionInOneRoundRPC (raft_etcd_paper_test.go:198-238): node 1 campaigns, the
    votes of the table arrive in the next step."""
    for i, c in enumerate(KATS["TestLeaderElectionInOneRoundRPC"]):
        votes = sorted((int(k), v) for k, v in c["votes"].items())
        steps = [[("campaign",)], [msg(VRESP, k, 2, reject=int(not v)) for k, v in votes]]
        yield dict(name=f"election{i}", group=(100 + i, 1, 1, FOLLOWER, 5, 5, 5,
                                               members(c["size"])),
                   steps=steps, want_state=c["want_state"], src=c["src"])


def candidate_vote_cases():
    """TestHandleCandidateRequestVoteResp(Rejected) (raft_test.go:2197-2239)."""
    for i, c in enumerate(KATS["TestHandleCandidateRequestVoteResp"]):
        steps = [[msg(VRESP, f, 2, reject=int(r)) for f, r in c["msgs"]]]
        yield dict(name=f"candvote{i}", group=(200 + i, 1, 2, CANDIDATE, 5, 5, 5,
                                               members(c["n"])),
                   steps=steps, want_state=c["want_state"], src=c["src"])


def check_quorum_cases():
    """TestHandleLeaderCheckQuorum / TestLeaderStepdownWhenQuorumActive/Lost (raft_test.go:
    1883-1900, raft_etcd_test.go:1610-1645): active flags -> leaderHasQuorum."""
    for i, c in enumerate(KATS["TestLeaderHasQuorum"]):
        steps = [[("check_quorum",)]]
        yield dict(name=f"checkq{i}", group=(300 + i, 1, 3, LEADER, 7, 8, 7,
                                             members(c["n"], c["active"])),
                   steps=steps, want_state=LEADER if c["want"] else FOLLOWER, src=c["src"])


def _term_start(case):
    log = {int(k): v for k, v in case["log"].items()}
    ts = case["last"] + 1
    for i in sorted(log, reverse=True):
        if log[i] != case["term"]:
            break
        ts = i
    # the step model needs a leader's log: monotone terms (entryutils.go:44-47), none above the
    # leader's term, every entry >= ts at the term
    mono = all(log[i] <= log[j] for i in log for j in log if i < j) and \
        max(log.values()) <= case["term"]
    return ts, mono


def commit_cases():
    """The commit tables of tests/golden (TestLeaderAcknowledgeCommit, TestLeaderOnlyCommits-
    LogFromCurrentTerm, TestLeaderCommitPrecedingEntries, TestCommitWithoutNewTermEntry,
    TestFullMemberWithOneWitness, TestLeaderAppResp, TestCommitAfterRemoveNode ...): the leader's
    followers report their match in ReplicateResp messages of one step."""
    k = 0
    for t in COMMIT_TABLES:
        for c in KATS[t]:
            ts, mono = _term_start(c)
            rem, wit = c["remotes"], c["witnesses"]
            if not mono or max(rem + wit) > c["last"] or c["committed"] > c["last"]:
                continue       # outside the step model (non-monotone log / ack beyond last)
            if rem[0] != c["last"]:
                continue       # slot 0 is the leader itself: its match is its lastIndex
            n = len(rem)
            wids = [n + 1 + j for j in range(len(wit))]
            mem = [(1, c["last"], REMOTE, 0)] + [(i + 1, 0, REMOTE, 0) for i in range(1, n)]
            mem += [(w, 0, WITNESS, 0) for w in wids]
            ms = [msg(RREP, i + 1, c["term"], rem[i]) for i in range(1, n) if rem[i] > 0]
            ms += [msg(RREP, wids[j], c["term"], wit[j]) for j in range(len(wit)) if wit[j] > 0]
            if not ms:
                ms = [("propose", 0)]   # single node: appendEntries is the tryCommit trigger
            yield dict(name=f"commit{k}", group=(400 + k, 1, c["term"], LEADER, c["committed"],
                                                 c["last"], ts, mem),
                       steps=[ms], want_committed=c["want_committed"], src=f"{t} {c['src']}")
            k += 1


def readindex_cases():
    """raft-level ReadIndex tests."""
    # TestLeaderReadIndexOnSingleNodeCluster (raft_test.go:2678-2702): campaign -> leader with
    # its no-op committed; the ReadIndex is ready at once with the committed index
    yield dict(name="ri_single", group=(501, 1, 0, FOLLOWER, 0, 0, 0, members(1)),
               steps=[[("campaign",)], [("read", 101, 1002)]],
               want_ready=[(1, 101, 1002)], want_pending=0, src="raft_test.go:2678-2702")
    # TestLeaderIgnoreReadIndexWhenClusterCommittedIsUnknown (raft_test.go:2704-2723)
    yield dict(name="ri_unknown", group=(502, 1, 0, FOLLOWER, 0, 0, 0, members(3)),
               steps=[[("campaign",)], [msg(VRESP, 2, 1)], [("read", 101, 1002)]],
               want_dropped=[(101, 1002, 0, D_NOT_READY)], want_pending=0,
               src="raft_test.go:2704-2723")
    # TestHandleLeaderReadIndex (raft_test.go:2725-2762): commit the no-op, then the request
    # is queued (pending 1)
    yield dict(name="ri_queue", group=(503, 1, 0, FOLLOWER, 0, 0, 0, members(3)),
               steps=[[("campaign",)], [msg(VRESP, 2, 1)], [msg(RREP, 2, 1, 1)],
                      [("read", 101, 1002)]],
               want_pending=1, src="raft_test.go:2725-2762")
    # TestWitnessReadIndex (raft_test.go:2764-2788): a witness' ReadIndex is dropped
    yield dict(name="ri_witness", group=(504, 1, 1, LEADER, 1, 1, 1,
                                         [(1, 1, REMOTE, 0), (2, 0, WITNESS, 0)]),
               steps=[[msg(READIDX, 2, 0, hint=101, high=1002)]],
               want_dropped=[(101, 1002, 2, D_WITNESS)], want_pending=0,
               src="raft_test.go:2764-2788")
    # TestObserverCanReadIndexQuorum1 (raft_test.go:458-497): single voter + observer 2; the
    # observer's ReadIndex is answered with the committed index
    yield dict(name="ri_observer", group=(505, 1, 1, LEADER, 11, 11, 1,
                                          [(1, 11, REMOTE, 0), (2, 0, OBSERVER, 0)]),
               steps=[[msg(READIDX, 2, 0, hint=12345)]],
               want_ready=[(11, 12345, 0)], want_resps=[(2, 11, 12345, 0)],
               src="raft_test.go:458-497")
    # readIndex.confirm prefix release with the index rewrite (readindex_test.go:125-162) and
    # the ReadIndexResp hint of handleReadIndexLeaderConfirmation (raft.go:1740-1760): ctx A
    # (from 2, index 3) and B (from 4, index 4 after the commit) are released together when B
    # reaches quorum; both answers carry B's index and B's ctx.
    yield dict(name="ri_prefix", group=(506, 1, 2, LEADER, 3, 5, 3,
                                        [(i, 5 if i == 1 else 3, REMOTE, 0)
                                         for i in range(1, 6)]),
               steps=[[msg(READIDX, 2, 2, hint=7, high=70),
                       msg(RREP, 2, 2, 4), msg(RREP, 3, 2, 4),
                       msg(READIDX, 4, 2, hint=8, high=80),
                       msg(HBRESP, 3, 2, hint=8, high=80), msg(HBRESP, 3, 2, hint=8, high=80),
                       msg(HBRESP, 5, 2, hint=8, high=80)]],
               want_committed=4, want_resps=[(2, 4, 8, 80), (4, 4, 8, 80)], want_pending=0,
               src="readindex_test.go:125-162, raft.go:1740-1760")
    yield _read_only_option_safe()
    # TestObserverCanReadIndexQuorum2 (raft_test.go:500-535): voters 1 (leader) and 2, observer
    # 3. Ten proposals; the observer's ReplicateResp alone commits nothing (observers are not
    # voting members, raft.go:888-909), node 2's commits all ten; the observer's ReadIndex is
    # forwarded to the leader, confirmed by node 2's heartbeat ack (observers never ack a ctx,
    # raft.go:843-847) and answered with the committed index.
    obs = [(1, 1, REMOTE, 0), (2, 1, REMOTE, 0), (3, 1, OBSERVER, 0)]
    yield dict(name="ri_observer2_noack", group=(507, 1, 1, LEADER, 1, 1, 1, obs),
               steps=[[("propose", 10)], [msg(RREP, 3, 1, 11)]], want_committed=1,
               src="raft_test.go:500-535")
    yield dict(name="ri_observer2", group=(508, 1, 1, LEADER, 1, 1, 1, obs),
               steps=[[("propose", 10)], [msg(RREP, 3, 1, 11)], [msg(RREP, 2, 1, 11)],
                      [msg(READIDX, 3, 1, hint=12345), msg(HBRESP, 2, 1, hint=12345)]],
               want_committed=11, want_resps=[(3, 11, 12345, 0)], want_pending=0,
               src="raft_test.go:500-535")
    # TestHasCommittedEntryAtCurrentTerm (raft_test.go:1863-1881): a new 2-voter leader has no
    # committed entry at its term until node 2 acks the no-op (hasCommittedEntryAtCurrentTerm,
    # raft.go:1612-1621), so a ReadIndex before that ack is dropped and one after it is queued
    yield dict(name="ri_committed_at_term", group=(509, 1, 0, FOLLOWER, 0, 0, 0, members(2)),
               steps=[[("campaign",)], [msg(VRESP, 2, 1)], [("read", 101, 1002)],
                      [msg(RREP, 2, 1, 1)], [("read", 103, 1004)]],
               want_state=LEADER, want_committed=1, want_dropped=[(101, 1002, 0, D_NOT_READY)],
               want_pending=1, src="raft_test.go:1863-1881")
    # TestReadIndexIsResetAfterRaftStateChange (readindex_test.go:164-175): a pending request
    # is dropped by reset() when a higher-term message turns the leader into a follower
    yield dict(name="ri_reset", group=(510, 1, 1, LEADER, 1, 1, 1,
                                       [(1, 1, REMOTE, 0), (2, 1, REMOTE, 0), (3, 1, REMOTE, 0)]),
               steps=[[("read", 10001, 10002)], [msg(HBRESP, 2, 2)]],
               want_state=FOLLOWER, want_pending=0, src="readindex_test.go:164-175")


def _read_only_option_safe():
    """TestReadOnlyOptionSafe (raft_etcd_test.go:1847-1899): leader 1 of voters {1, 2, 3} at term
    1 with its no-op committed. Six rounds of ten proposals, each committed by both followers'
    acks, then a ReadIndex at node 1 (local), 2 or 3 (forwarded to the leader), confirmed by the
    heartbeat acks: the read index is the committed index 11, 21, ..., 61 with the request's ctx
    (getTestSystemCtx(v) = {v, v + 1}, readindex_test.go:23-28); a follower's read comes back
    as the ReadIndexResp of raft.go:1751-1757."""
    table = [(1, 11, 10001), (2, 21, 10002), (3, 31, 10003),
             (1, 41, 10004), (2, 51, 10005), (3, 61, 10006)]
    steps, ready, resps = [], [], []
    for who, wri, v in table:
        steps.append([("propose", 10)])
        steps.append([msg(RREP, 2, 1, wri), msg(RREP, 3, 1, wri)])
        acks = [msg(HBRESP, 2, 1, hint=v, high=v + 1), msg(HBRESP, 3, 1, hint=v, high=v + 1)]
        if who == 1:
            steps.append([("read", v, v + 1)] + acks)
            ready.append((wri, v, v + 1))
        else:
            steps.append([msg(READIDX, who, 1, hint=v, high=v + 1)] + acks)
            resps.append((who, wri, v, v + 1))
    return dict(name="ri_read_only_safe", group=(511, 1, 1, LEADER, 1, 1, 1,
                                                 [(i, 1, REMOTE, 0) for i in (1, 2, 3)]),
                steps=steps, want_committed=61, want_ready=ready, want_resps=resps,
                want_pending=0, src="raft_etcd_test.go:1847-1899")


def single_node_commit_cases():
    """TestSingleNodeCommit (raft_etcd_test.go:697-707): proposals commit at once."""
    yield dict(name="single_commit", group=(601, 1, 1, LEADER, 1, 1, 1, members(1)),
               steps=[[("propose", 1), ("propose", 1)]], want_committed=3,
               src="raft_etcd_test.go:697-707")


def all_cases():
    for f in (election_cases, candidate_vote_cases, check_quorum_cases, commit_cases,
              readindex_cases, single_node_commit_cases):
        yield from f()


def run_case(backend, case):
    """Runs a scenario; returns (outputs of every step, final state)."""
    cid = case["group"][0]
    backend.add_group(*case["group"])
    outs = [backend.step({cid: ev}) for ev in case["steps"]]
    return [o[cid] for o in outs], backend.state(cid)


def check_case(case, outs, state):
    term, st, committed, last, ts, mem, reads = state
    if "want_state" in case:
        assert st == case["want_state"], (case["name"], case["src"], st)
    if "want_committed" in case:
        assert committed == case["want_committed"], (case["name"], case["src"], committed)
    if "want_pending" in case:
        assert len(reads) == case["want_pending"], (case["name"], reads)
    ready = [r for o in outs for r in o["ready"]]
    resps = [r for o in outs for r in o["resps"]]
    dropped = [r for o in outs for r in o["dropped"]]
    if "want_ready" in case:
        assert ready == case["want_ready"], (case["name"], ready)
    if "want_resps" in case:
        assert resps == case["want_resps"], (case["name"], resps)
    if "want_dropped" in case:
        assert dropped == case["want_dropped"], (case["name"], dropped)
