#!/usr/bin/env python3
"""Writes tests/golden/reference_kats.json: known-answer vectors of the reference's own tests.

Every table below is transcribed by hand from dragonboat's Go tests (the reference at
/root/reference; paths relative to it). The Go toolchain is absent from this image, so the
reference cannot be executed; these tables are what pins the CPU oracle (oracle/qref.c). Tables
marked "derived" reduce a network-level test (internal/raft/raft_etcd_test.go `network`) to the
inputs that reach the quorum arithmetic at the checked point; the derivation is in `note`.

Run: python tests/golden/make_golden.py   (rewrites reference_kats.json deterministically)
"""
import json
import os

OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "reference_kats.json")


def commit_case(src, remotes, witnesses, log, term, committed, want, first_minus_1=0, note=""):
    """One raft.tryCommit call: `log` maps index -> term for [first_minus_1, last]."""
    return {
        "src": src,
        "remotes": remotes,
        "witnesses": witnesses,
        "first_minus_1": first_minus_1,
        "last": max(log) if log else first_minus_1,
        "log": {str(k): v for k, v in sorted(log.items())},
        "term": term,
        "committed": committed,
        "want_committed": want,
        "note": note,
    }


def kats():
    out = {}

    # ---- TestCommit — internal/raft/raft_etcd_test.go:1111-1160 ---------------------------
    # newTestRaft(1,[1]) + setRemote(j+1, matches[j]); storage state Term = smTerm; the
    # TestLogDB marker entry is index 0 term 0 (logdb_test.go:98-101).
    T = [
        ([1], [(1, 1)], 1, 1),
        ([1], [(1, 1)], 2, 0),
        ([2], [(1, 1), (2, 2)], 2, 2),
        ([1], [(1, 2)], 2, 1),
        ([2, 1, 1], [(1, 1), (2, 2)], 1, 1),
        ([2, 1, 1], [(1, 1), (2, 1)], 2, 0),
        ([2, 1, 2], [(1, 1), (2, 2)], 2, 2),
        ([2, 1, 2], [(1, 1), (2, 1)], 2, 0),
        ([2, 1, 1, 1], [(1, 1), (2, 2)], 1, 1),
        ([2, 1, 1, 1], [(1, 1), (2, 1)], 2, 0),
        ([2, 1, 1, 2], [(1, 1), (2, 2)], 1, 1),
        ([2, 1, 1, 2], [(1, 1), (2, 1)], 2, 0),
        ([2, 1, 2, 2], [(1, 1), (2, 2)], 2, 2),
        ([2, 1, 2, 2], [(1, 1), (2, 1)], 2, 0),
    ]
    out["TestCommit"] = [
        commit_case(f"raft_etcd_test.go:1118-1136 #{i}", m, [], {0: 0, **dict(logs)}, sm, 0, w)
        for i, (m, logs, sm, w) in enumerate(T)
    ]

    # ---- TestLeaderOnlyCommitsLogFromCurrentTerm — raft_etcd_paper_test.go:854-885 --------
    # ents {1:t1, 2:t2}; loadState(Term 2) -> becomeCandidate (term 3) -> becomeLeader appends
    # the no-op at index 3 (term 3); Propose -> index 4 (term 3); ReplicateResp from 2 with
    # LogIndex = index: matched = {self: 4, node 2: index}.
    out["TestLeaderOnlyCommitsLogFromCurrentTerm"] = [
        commit_case(f"raft_etcd_paper_test.go:860-866 #{i}", [4, idx], [],
                    {0: 0, 1: 1, 2: 2, 3: 3, 4: 3}, 3, 0, want)
        for i, (idx, want) in enumerate([(1, 0), (2, 0), (3, 3)])
    ]

    # ---- TestLeaderAcknowledgeCommit — raft_etcd_paper_test.go:448-483 (derived) -----------
    # leader term 1; commitNoopEntry (:925-948) makes every follower accept the no-op
    # (match 1, committed 1); Propose -> index 2; acceptors reply match 2.
    AC = [
        (1, [], True), (3, [], False), (3, [2], True), (3, [2, 3], True),
        (5, [], False), (5, [2], False), (5, [2, 3], True), (5, [2, 3, 4], True),
        (5, [2, 3, 4, 5], True),
    ]
    cases = []
    for i, (size, acc, wack) in enumerate(AC):
        matches = [2] + [2 if nid in acc else 1 for nid in range(2, size + 1)]
        cases.append(commit_case(f"raft_etcd_paper_test.go:454-464 #{i}", matches, [],
                                 {0: 0, 1: 1, 2: 1}, 1, 1, 2 if wack else 1,
                                 note="committed > li(=1) iff wack"))
    out["TestLeaderAcknowledgeCommit"] = cases

    # ---- TestLeaderCommitPrecedingEntries — raft_etcd_paper_test.go:490-518 (derived) ------
    # loadState(Term 2) -> term 3 leader; no-op at li+1, proposal at li+2 (term 3); all accept.
    pre = [[], [(1, 2)], [(1, 1), (2, 2)], [(1, 1)]]
    cases = []
    for i, ents in enumerate(pre):
        li = len(ents)
        log = {0: 0, **dict(ents), li + 1: 3, li + 2: 3}
        cases.append(commit_case(f"raft_etcd_paper_test.go:491-496 #{i}", [li + 2] * 3, [], log,
                                 3, 0, li + 2, note="every preceding entry committed"))
    out["TestLeaderCommitPrecedingEntries"] = cases

    # ---- TestSingleNodeCommit / Cannot/CommitWithoutNewTermEntry (derived) -----------------
    out["TestSingleNodeCommit"] = [
        commit_case("raft_etcd_test.go:697-707", [3], [], {0: 0, 1: 1, 2: 1, 3: 1}, 1, 1, 3),
    ]
    # 5 nodes; node 1 (term 1) wrote no-op 1 + proposals 2,3 but reached only node 2; node 2
    # becomes leader at term 2 and appends its no-op at index 4.
    log5 = {0: 0, 1: 1, 2: 1, 3: 1, 4: 2}
    out["TestCannotCommitWithoutNewTermEntry"] = [
        commit_case("raft_etcd_test.go:734-743", [4, 0, 0, 0, 0], [], log5, 2, 1, 1,
                    note="Replicate ignored: only the leader holds index 4"),
        commit_case("raft_etcd_test.go:734-743", [4, 3, 1, 1, 1], [], log5, 2, 1, 1,
                    note="old-term entries are never committed by counting replicas"),
        commit_case("raft_etcd_test.go:745-754", [5, 5, 5, 5, 5], [],
                    {**log5, 5: 2}, 2, 1, 5, note="a current-term entry commits everything"),
    ]
    out["TestCommitWithoutNewTermEntry"] = [
        commit_case("raft_etcd_test.go:775-783", [4, 4, 4, 4, 4], [], log5, 2, 1, 4),
    ]

    # ---- TestLeaderAppResp — raft_etcd_test.go:1901-1946 (tryCommit part) -------------------
    # logdb {1:t0, 2:t1}, inmem marker 3; leader term 1 appends no-op at 3; remote 2 ReplicateResp
    out["TestLeaderAppResp"] = [
        commit_case("raft_etcd_test.go:1914 accept 2", [3, 2, 0], [], {0: 0, 1: 0, 2: 1, 3: 1},
                    1, 0, 2),
        commit_case("raft_etcd_test.go:1915 heartbeat reply", [3, 0, 0], [],
                    {0: 0, 1: 0, 2: 1, 3: 1}, 1, 0, 0),
    ]

    # ---- witnesses count toward the commit quorum ------------------------------------------
    # TestFullMemberWithOneWitnessCouldMakeProgressWithOneMemberDrop — raft_test.go:1627-1662:
    # 3 full + 1 witness (n = 4, quorum 3); node 3 isolated after the second entry.
    out["TestFullMemberWithOneWitness"] = [
        commit_case("raft_test.go:1644-1651", [2, 2, 2], [2], {0: 0, 1: 1, 2: 1}, 1, 1, 2),
        commit_case("raft_test.go:1653-1661", [3, 3, 2], [3], {0: 0, 1: 1, 2: 1, 3: 1}, 1, 2, 3,
                    note="isolated full member lags; the witness completes the quorum"),
    ]
    # TestVotingMemberLengthMismatchWillResetMatchArray — raft_test.go:2790-2808
    out["TestVotingMemberLengthMismatch"] = [
        commit_case("raft_test.go:2791-2806", [1, 1, 0], [0], {0: 0, 1: 1}, 1, 0, 0,
                    note="witness 4 added after the no-op: n = 4, quorum 3 -> no commit"),
    ]
    # TestCommitAfterRemoveNode — raft_etcd_test.go:2611-2668 (derived). Two voters; leader at
    # term 1 writes its no-op (1), the RemoveNode entry (2) and "hello" (3). Node 2 acks the
    # config change: matched {self 3, node 2: 2} -> 2 commits, entries 1-2 ("two committed
    # entries", :2653-2656). removeNode(2) re-runs tryCommit over the one remaining voter
    # (raft.go:1194-1198): q = 3 commits "hello" (:2666-2671).
    log_rm = {0: 0, 1: 1, 2: 1, 3: 1}
    out["TestCommitAfterRemoveNode"] = [
        commit_case("raft_etcd_test.go:2646-2656", [3, 2], [], log_rm, 1, 0, 2,
                    note="node 2 acks the config-change entry"),
        commit_case("raft_etcd_test.go:2663-2671", [3], [], log_rm, 1, 2, 3,
                    note="after removeNode(2): one voter, quorum 1"),
    ]
    # TestCommitTo — logentry_etcd_test.go:374-406 (derived): previous entries {1:t1, 2:t2,
    # 3:t3}, committed 2. commitTo(3) -> 3; commitTo(1) -> 2 (never decreases); commitTo(4)
    # panics, which tryCommit never reaches: an index above lastIndex has term 0
    # (logentry.go:144-147), so q = 4 fails the term check and committed stays 2.
    log_ct = {0: 0, 1: 1, 2: 2, 3: 3}
    out["TestCommitTo"] = [
        commit_case("logentry_etcd_test.go:379", [3], [], log_ct, 3, 2, 3),
        commit_case("logentry_etcd_test.go:380", [3, 1, 1], [], log_ct, 3, 2, 2,
                    note="q = 1 <= committed: never decrease"),
        commit_case("logentry_etcd_test.go:381", [3, 4, 4], [], log_ct, 3, 2, 2,
                    note="q = 4 > lastIndex: term(4) = 0, the commitTo panic is unreachable"),
    ]
    # TestTryCommitResetsMatchArray — raft_test.go:136-145 (derived): a fresh 3-voter leader at
    # term 1 (no-op at 1, no acks): tryCommit sizes matched to 3 voters; q = 0, nothing commits
    out["TestTryCommitResetsMatchArray"] = [
        commit_case("raft_test.go:137-144", [1, 0, 0], [], {0: 0, 1: 1}, 1, 0, 0),
    ]

    # ---- sortMatchValues / quorum — raft_test.go:2033-2055, :1525-1549 ---------------------
    out["TestUnrolledBubbleSortMatchValue"] = [
        {"src": "raft_test.go:2036-2043", "vals": v, "want": sorted(v)}
        for v in ([1, 1, 1], [1, 1, 2], [1, 2, 2], [2, 3, 1], [3, 2, 1], [3, 3, 1])
    ]
    out["TestQuorumValue"] = [
        {"src": "raft_test.go:1525-1538", "n": n, "quorum": q} for n, q in ((1, 1), (2, 2), (5, 3))
    ]
    out["TestIsSingleNodeQuorum"] = [
        {"src": "raft_test.go:1540-1549", "n": n, "single": s} for n, s in ((1, True), (3, False))
    ]

    # ---- entryLog.term — logentry_etcd_test.go:566-629, inmemory_test.go:164-224 -----------
    off, num = 100, 100
    log = {off: 1, **{off + i: i for i in range(1, num)}}
    out["TestTerm"] = [
        {"src": "logentry_etcd_test.go:580-586", "first_minus_1": off, "last": off + num - 1,
         "log": {str(k): v for k, v in log.items()}, "index": i, "want": w}
        for i, w in ((off - 1, 0), (off, 1), (off + num // 2, num // 2), (off + num - 1, num - 1),
                     (off + num, 0))
    ]
    out["TestTermWithUnstableSnapshot"] = [
        {"src": "logentry_etcd_test.go:610-620", "first_minus_1": 105, "last": 105,
         "log": {"105": 1}, "index": i, "want": w}
        for i, w in ((100, 0), (101, 0), (104, 0), (105, 1))
    ]
    out["TestInMemGetTerm"] = [
        {"src": "inmemory_test.go:207-211", "first_minus_1": 100, "last": 104,
         "log": {str(i): i for i in range(100, 105)}, "index": i, "want": w}
        for i, w in ((103, 103), (104, 104), (105, 0))
    ]
    out["TestInMemGetTermReturnSnapshotTerm"] = [
        {"src": "inmemory_test.go:173-176", "first_minus_1": 5, "last": 5, "log": {"5": 2},
         "index": i, "want": w}
        for i, w in ((5, 2), (4, 0), (10, 0))
    ]

    # ---- readIndex — readindex_test.go ------------------------------------------------------
    def ctx(v):  # getTestSystemCtx (readindex_test.go:21-26)
        return [v, v + 1]

    out["TestReadIndexLeaderCanBeConfirmed"] = {
        "src": "readindex_test.go:125-162",
        "ops": [
            ["add", 3, ctx(10002), 1], ["add", 4, ctx(10001), 3], ["add", 5, ctx(10003), 2],
            ["confirm", ctx(10001), 1, 3, None],
            ["confirm", ctx(10001), 3, 3, [[4, 1, ctx(10002)], [4, 3, ctx(10001)]]],
        ],
        "final_pending": 1, "final_queue": 1,
    }
    out["TestSameCtxCanNotBeAddedTwice"] = {
        "src": "readindex_test.go:30-40",
        "ops": [["add", 1, ctx(10001), 1], ["add", 2, ctx(10001), 2]],
        "final_pending": 1, "final_queue": 1,
    }
    out["TestReadIndexRequestCanBeAdded"] = {
        "src": "readindex_test.go:56-82",
        "ops": [["add", 1, ctx(10001), 1], ["add", 2, ctx(10002), 2]],
        "final_pending": 2, "final_queue": 2,
    }
    out["TestReadIndexChecksInputIndex"] = {
        "src": "readindex_test.go:84-102",
        "ops": [["add", 3, ctx(10001), 1], ["add", 5, ctx(10002), 3],
                ["add_panics", 4, ctx(10003), 2]],
    }

    # ---- votes -------------------------------------------------------------------------------
    out["TestHandleVoteResp"] = {
        "src": "raft_test.go:1710-1719",
        "seq": [[1, False, 1], [2, True, 1], [3, False, 2], [2, False, 2]],
    }
    # TestLeaderElectionInOneRoundRPC — raft_etcd_paper_test.go:198-238
    LE = [
        (1, {}, 2), (3, {2: True, 3: True}, 2), (3, {2: True}, 2),
        (5, {2: True, 3: True, 4: True, 5: True}, 2), (5, {2: True, 3: True, 4: True}, 2),
        (5, {2: True, 3: True}, 2),
        (3, {2: False, 3: False}, 0), (5, {2: False, 3: False, 4: False, 5: False}, 0),
        (5, {2: True, 3: False, 4: False, 5: False}, 0),
        (3, {}, 1), (5, {2: True}, 1), (5, {2: False, 3: False}, 1), (5, {}, 1),
    ]
    out["TestLeaderElectionInOneRoundRPC"] = [
        {"src": f"raft_etcd_paper_test.go:205-224 #{i}", "size": size,
         "votes": {str(k): v for k, v in votes.items()}, "want_state": st}
        for i, (size, votes, st) in enumerate(LE)
    ]
    # TestHandleCandidateRequestVoteResp(Rejected) — raft_test.go:2197-2239 (no self vote:
    # becomeCandidate only)
    out["TestHandleCandidateRequestVoteResp"] = [
        {"src": "raft_test.go:2197-2218", "n": 3,
         "msgs": [[1, False], [2, False], [3, False]], "want_state": 2},
        {"src": "raft_test.go:2220-2239", "n": 3, "msgs": [[2, True], [3, True]],
         "want_state": 0},
    ]

    # ---- CheckQuorum — raft_test.go:1883-1900, raft_etcd_test.go:1610-1645 ------------------
    out["TestLeaderHasQuorum"] = [
        {"src": "raft_test.go:1884-1889", "n": 2, "active": [False, False], "want": False},
        {"src": "raft_test.go:1890-1899", "n": 2, "active": [True, True], "want": True},
        {"src": "raft_etcd_test.go:1610-1627", "n": 3, "active": [False, True, False],
         "want": True},
        {"src": "raft_etcd_test.go:1629-1645", "n": 3, "active": [False, False, False],
         "want": False},
    ]
    return out


def main():
    with open(OUT, "w") as f:
        json.dump(kats(), f, indent=1, sort_keys=True)
        f.write("\n")
    print("wrote", OUT)


if __name__ == "__main__":
    main()
