"""Random groups and per-step event streams for the step-worker differential tests. Streams stay
inside the worker's contract (no observer acking a pending ctx, no ReplicateResp above the
leader's lastIndex, at most 8 pending ReadIndex ctxs) so every event is decided, and cover
everything else: witnesses, observers, non-members, stale / zero / higher terms, duplicate
acks, several ReadIndex ctxs per group, mid-step ReadIndex after commits, campaigns, CheckQuorum
and proposals."""
import numpy as np

import step_scenarios as sc


def random_groups(rng, G, cid0=1):
    groups = []
    for j in range(G):
        n_rem = int(rng.choice([1, 2, 3, 3, 3, 4, 5, 5, 5, 6, 7, 8]))
        n_wit = int(rng.integers(0, 3)) if n_rem + 2 <= 8 and n_rem >= 2 else 0
        n_obs = int(rng.integers(0, 3))
        ids = rng.choice(np.arange(1, 64), n_rem + n_wit + n_obs, replace=False)
        roles = [sc.REMOTE] * n_rem + [sc.WITNESS] * n_wit + [sc.OBSERVER] * n_obs
        node = int(ids[0])
        state = int(rng.choice([sc.LEADER] * 6 + [sc.CANDIDATE] * 2 + [sc.FOLLOWER] * 2))
        term = int(rng.integers(2, 9))
        last = 100 + int(rng.integers(0, 50))
        term_start = last - int(rng.integers(0, 6))
        committed = last - int(rng.integers(0, 9))
        mem = []
        for i, r in zip(ids, roles):
            i = int(i)
            if i == node:
                m = last
            elif state == sc.LEADER:
                m = int(rng.integers(max(0, committed - 3), last + 1))
            else:
                m = 0
            mem.append((i, m, r, int(rng.random() < 0.5)))
        order = rng.permutation(len(mem))
        mem = [mem[k] for k in order]
        groups.append((cid0 + j, node, term, state, committed, last, term_start, mem,
                       random_log(rng, term, state, committed, term_start)))
    return groups


def random_log(rng, term, state, committed, term_start):
    """A multi-term log history for the oracle (qref_group_set_log): 1-4 runs of older terms
    below term_start (run 0 from index 0), then term_start's run at the group's term (a
    candidate's at term - 1: it has no entries of the term it campaigns in), and a compaction
    point at or below committed (term 0 below it, logentry.go:143-160)."""
    top = term - 1 if state == sc.CANDIDATE else term
    k = int(rng.integers(1, min(4, top - 1) + 1)) if top > 1 else 0
    terms = sorted(int(t) for t in rng.choice(np.arange(1, top), k, replace=False)) if k else []
    starts = [0] + sorted(int(x) for x in rng.choice(np.arange(1, max(2, term_start)),
                                                     min(k - 1, max(0, term_start - 1)),
                                                     replace=False)) if k else []
    terms = terms[:len(starts)]
    runs = list(zip(starts, terms))
    if not runs:                 # a candidate at term 2: every entry at term 1
        runs = [(0, top)]
    elif term_start > starts[-1]:
        runs.append((term_start, top))
    first_minus_1 = max(0, committed - int(rng.integers(0, 40)))
    return first_minus_1, runs


def random_events(rng, state, step_no, ctx_seq):
    """One step of events for a group whose state (backend.state()) is `state`."""
    term, st, committed, last, ts, mem, reads = state
    ids = [m[0] for m in mem]
    role = {m[0]: m[2] for m in mem}
    ctxs = [r[2] for r in reads]
    cap = 8 - len(reads)
    ev = []

    def new_ctx():
        ctx_seq[0] += 1
        return (ctx_seq[0], step_no)

    if rng.random() < 0.3 and cap > 0:                           # node.handleReadIndex
        c = new_ctx()
        ctxs.append(c)
        cap -= 1
        ev.append(("read", c[0], c[1]))
    for _ in range(int(rng.integers(0, 14))):                    # handleReceivedMessages
        frm = int(rng.choice(ids)) if rng.random() > 0.05 else 999
        u = rng.random()
        mterm = term if u < 0.8 else 0 if u < 0.88 else term - 1 if u < 0.97 else term + 1
        r = rng.random()
        if r < 0.35:
            idx = int(rng.integers(max(0, last - 6), last + 1))
            ev.append(sc.msg(sc.RREP, frm, mterm, idx, reject=int(rng.random() < 0.1)))
        elif r < 0.72:
            hint = high = 0
            if ctxs and rng.random() < 0.85 and role.get(frm) != sc.OBSERVER:
                hint, high = ctxs[int(rng.integers(0, len(ctxs)))]
            ev.append(sc.msg(sc.HBRESP, frm, mterm, hint=hint, high=high))
        elif r < 0.88:
            ev.append(sc.msg(sc.VRESP, frm, mterm, reject=int(rng.random() < 0.35)))
        elif cap > 0:
            c = new_ctx() if rng.random() > 0.1 or not ctxs else ctxs[0]
            if c not in ctxs:
                ctxs.append(c)
                cap -= 1
            ev.append(sc.msg(sc.READIDX, frm, mterm, hint=c[0], high=c[1]))
    if st == sc.LEADER and rng.random() < 0.15:                  # handleLocalTick
        ev.append(("check_quorum",))
    if st != sc.LEADER and rng.random() < 0.25:
        ev.append(("campaign",))
    if rng.random() < 0.3:                                       # handleProposals
        ev.append(("propose", int(rng.integers(0, 4))))
    return ev
