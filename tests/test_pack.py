"""Membership roles end to end: fleets of groups with remotes, witnesses and observers (non-voting
members), packed by the C++ packers of libhipquorum.so (hq_pack_*), decided by the oracle's batch
form on CPU and by the kernels on GPU, and compared with the oracle's role-aware scalar
restatement (tryCommit iterating r.remotes then r.witnesses, raft.go:888-909; votes with the
Peer.Handle / observer filters, peer.go:186-198, raft.go:1968-1985; readIndex.confirm;
leaderHasQuorum over votingMembers, raft.go:380-390)."""
import numpy as np
import pytest

from dragonboat_amd import hipquorum as hq
from oracle import qref

ROLE_R, ROLE_O, ROLE_W = hq.ROLE_REMOTE, hq.ROLE_OBSERVER, hq.ROLE_WITNESS


def make_fleet(seed, G, with_msgs=True, big=True):
    """Random leader/candidate groups. Returns (groups, members, msgs, truth) where truth keeps
    the role-aware view each group's reference raft struct would hold."""
    rng = np.random.default_rng(seed)
    groups = np.zeros(G, hq.GROUP_DTYPE)
    mem, msgs, truth = [], [], []
    for g in range(G):
        nr = int(rng.integers(1, 7))
        nw = int(rng.integers(0, 3))
        no = int(rng.integers(0, 4))
        if big and g % 53 == 0:
            nr, nw = 7, 2                     # 9 voting members: beyond n_max -> fallback
        ids = rng.choice(np.arange(1, 5000), nr + nw + no, replace=False).astype(np.uint64)
        roles = [ROLE_R] * nr + [ROLE_W] * nw + [ROLE_O] * no
        order = rng.permutation(len(ids))
        self_id = int(ids[rng.integers(0, nr)])
        if g % 61 == 7:
            self_id = 999_999                  # own node missing from the remotes -> fallback
        last = int(rng.integers(30, 60))
        committed = last - int(rng.integers(0, 10))
        term_start = committed - int(rng.integers(-3, 4))
        term = 5
        view = dict(remotes={}, witnesses={}, observers={}, self=self_id, last=last,
                    committed=committed, term_start=term_start, term=term, active={})
        first = len(mem)
        for j in order:
            nid, role = int(ids[j]), roles[j]
            match = max(0, committed - int(rng.integers(0, 6)) + int(rng.integers(0, 12)))
            if nid == self_id:
                match = last
            active = int(rng.random() < 0.5)
            mem.append((nid, match, role, active))
            {ROLE_R: view["remotes"], ROLE_W: view["witnesses"], ROLE_O: view["observers"]}[role][nid] = match
            view["active"][nid] = active
        mask = 0
        for i in range(last - 15, last + 1):
            mask |= int(i >= term_start) << (i % 16)
        ctx = (int(rng.integers(1, 1 << 62)), int(rng.integers(1, 1 << 62)))
        first_msg = len(msgs)
        if with_msgs:
            senders = list(ids) + [np.uint64(777_777)]       # + a non-member
            for _ in range(int(rng.integers(0, 12))):
                frm = int(senders[rng.integers(0, len(senders))])
                is_obs = frm in view["observers"]
                hint = ctx if (rng.random() < 0.7 and not is_obs) else (ctx[0] + 1, ctx[1])
                msgs.append((frm, hint[0], hint[1], int(rng.random() < 0.35), 0))
        groups[g] = (self_id, committed, last, term_start, term, ctx[0], ctx[1], mask, 0, 0,
                     first, len(mem) - first, first_msg, len(msgs) - first_msg)
        view["ctx"] = ctx
        view["msgs"] = msgs[first_msg:]
        truth.append(view)
    members = np.array(mem, dtype=hq.MEMBER_DTYPE)
    msgs_a = np.array(msgs if msgs else [(0, 0, 0, 0, 0)], dtype=hq.MSG_DTYPE)
    return groups, members, msgs_a, truth


def packable(v):
    return v["self"] in v["remotes"] and len(v["remotes"]) + len(v["witnesses"]) <= 8


def ref_commit(v):
    terms = {i: (v["term"] if i >= v["term_start"] else v["term"] - 1)
             for i in range(v["committed"], v["last"] + 1)}
    log = qref.EntryLog(v["committed"], v["last"], v["committed"], terms)
    qref.try_commit(list(v["remotes"].values()), list(v["witnesses"].values()), log, v["term"])
    return log.committed


def ref_vote(v):
    n = len(v["remotes"]) + len(v["witnesses"])
    q = qref.quorum(n)
    votes = qref.PyVotes()
    votes.handle_vote_resp(v["self"], False)               # campaign, raft.go:1093
    state = qref.QREF_LEADER if q == 1 else qref.QREF_CANDIDATE
    members = set(v["remotes"]) | set(v["witnesses"]) | set(v["observers"])
    for frm, _, _, rej, _ in v["msgs"]:
        if state != qref.QREF_CANDIDATE:
            break
        if frm not in members:                              # Peer.Handle drops it
            continue
        state = votes.candidate_resp(frm, bool(rej), frm in v["observers"], q)
    return state


def ref_readindex(v):
    n = len(v["remotes"]) + len(v["witnesses"])
    q = qref.quorum(n)
    if q == 1:
        return True                                         # raft.go:1655-1667
    ri = qref.PyReadIndex()
    ri.add_request(v["committed"], v["ctx"], v["self"])
    members = set(v["remotes"]) | set(v["witnesses"]) | set(v["observers"])
    ok = False
    for frm, hl, hh, _, _ in v["msgs"]:
        if frm in members and (hl, hh) != (0, 0):
            ok |= ri.confirm((hl, hh), frm, q) is not None
    return ok


def ref_check_quorum(v):
    voting = list(v["remotes"]) + list(v["witnesses"])
    ids = np.array(voting, np.uint64)
    act = np.array([v["active"][i] for i in voting], np.int32)
    return bool(qref.lib.qref_leader_has_quorum(ids.ctypes.data, act.ctypes.data, len(voting),
                                                 v["self"]))


def test_pack_commit_matches_role_aware_oracle_on_cpu():
    groups, members, _, truth = make_fleet(11, 3000, with_msgs=False)
    cols, fb = hq.pack_commit(groups, members, 8)
    out = np.zeros(len(groups), np.uint64)
    ofb = np.zeros_like(fb)
    a = qref.commit_args(len(groups), 8, 0, 16, cols["match"], cols["committed_in"], out,
                         cols["last_index"], term_start=cols["term_start"],
                         n_voting=cols["n_voting"], fallback=ofb)
    assert qref.commit_batch(a, 4) == 0
    np.testing.assert_array_equal(fb, ofb)     # packing fallbacks surface as kernel fallbacks
    for g, v in enumerate(truth):
        if packable(v):
            assert not (fb[g >> 6] >> np.uint64(g & 63)) & np.uint64(1)
            assert out[g] == ref_commit(v), g
        else:
            assert (fb[g >> 6] >> np.uint64(g & 63)) & np.uint64(1)
            assert cols["n_voting"][g] == 0
    # observers never reach a slot: voter counts equal remotes + witnesses
    for g, v in enumerate(truth):
        if packable(v):
            assert cols["n_voting"][g] == len(v["remotes"]) + len(v["witnesses"])
            assert cols["match"][g] == v["remotes"][v["self"]]   # slot 0 = the leader


def test_pack_votes_and_acks_match_role_aware_oracle_on_cpu():
    groups, members, msgs, truth = make_fleet(12, 2000)
    gr, rj, nv, fb = hq.pack_votes(groups, members, msgs)
    out, _ = qref.vote_batch(gr, rj, nv, 0)
    ack, act, nv2, fb2 = hq.pack_acks(groups, members, msgs)
    conf, _ = qref.readindex_batch(ack, nv2, 0)
    hqb, _, _ = qref.check_quorum_batch(act, nv2, 0, 0)
    np.testing.assert_array_equal(fb, fb2)
    for g, v in enumerate(truth):
        if not packable(v):
            continue
        assert (int(out[g >> 5]) >> (2 * (g & 31))) & 3 == ref_vote(v), g
        assert bool((int(conf[g >> 6]) >> (g & 63)) & 1) == ref_readindex(v), g
        assert bool((int(hqb[g >> 6]) >> (g & 63)) & 1) == ref_check_quorum(v), g


@pytest.mark.gpu
def test_packed_fleet_through_the_kernels(gpu_ctx):
    groups, members, msgs, truth = make_fleet(13, 20_000)
    G = len(groups)
    cols, fb = hq.pack_commit(groups, members, 8)
    for form in (hq.HQ_FORM_TERM_START, hq.HQ_FORM_TERM_MASK):
        out = np.zeros(G, np.uint64)
        chg = np.zeros(hq.words64(G), np.uint64)
        kfb = np.zeros(hq.words64(G), np.uint64)
        a = hq.CommitArgs()
        a.G, a.n_max, a.form, a.ring_len, a.match_stride = G, 8, form, 16, G
        for k in ("match", "n_voting", "committed_in", "last_index", "term_start", "term_mask"):
            setattr(a, k, cols[k].ctypes.data)
        a.committed_out, a.changed, a.fallback = out.ctypes.data, chg.ctypes.data, kfb.ctypes.data
        gpu_ctx.commit_host(a)
        np.testing.assert_array_equal(kfb, fb)
        want = np.array([ref_commit(v) if packable(v) else v["committed"] for v in truth], np.uint64)
        np.testing.assert_array_equal(out, want)
    gr, rj, nv, _ = hq.pack_votes(groups, members, msgs)
    outc = np.zeros(hq.words32(G), np.uint64)
    gpu_ctx.vote_host(G, gr, rj, nv, 0, outc)
    ack, act, nv2, _ = hq.pack_acks(groups, members, msgs)
    conf = np.zeros(hq.words64(G), np.uint64)
    gpu_ctx.readindex_host(G, ack, nv2, 0, conf)
    da, dn = gpu_ctx.upload(act), gpu_ctx.upload(nv2)
    hqb = gpu_ctx.empty(hq.words64(G), np.uint64)
    gpu_ctx.check_quorum_dev(G, da, dn, 0, 0, hqb)
    hqh = gpu_ctx.download(hqb)
    for g, v in enumerate(truth):
        if not packable(v):
            continue
        assert (int(outc[g >> 5]) >> (2 * (g & 31))) & 3 == ref_vote(v), g
        assert bool((int(conf[g >> 6]) >> (g & 63)) & 1) == ref_readindex(v), g
        assert bool((int(hqh[g >> 6]) >> (g & 63)) & 1) == ref_check_quorum(v), g
    for x in (da, dn, hqb):
        gpu_ctx.free(x)
