"""Shared driver for step-level tests: the same per-group event streams run through the CPU oracle
(oracle/qref_step.c, one event at a time as the reference does) or through the GPU step worker
(hq_worker_step), with results split per group in one format.

An event is a tuple, listed per group in node.handleEvents order (node.go:1113-1157):
  ("read", ctx_low, ctx_high)                                     local ReadIndex
  ("msg", type, from, term, log_index, hint, hint_high, reject)    received message
  ("check_quorum",) / ("campaign",)                                tick messages
  ("propose", n_entries)                                           proposal
"""
import numpy as np

PHASE = {"read": 0, "msg": 1, "check_quorum": 2, "campaign": 2, "propose": 3}


def check_phase_order(events):
    ph = [PHASE[e[0]] for e in events]
    assert ph == sorted(ph), events


def event_record(hq, e):
    """An event tuple as an hq_event record (kind, type, from, term, log_index, hint,
    hint_high, reject, reserved)."""
    k = e[0]
    if k == "read":
        return (hq.EV_READ, 0, 0, 0, 0, e[1], e[2], 0, 0)
    if k == "msg":
        return (hq.EV_MESSAGE, e[1], e[2], e[3], e[4], e[5], e[6], e[7], 0)
    if k == "check_quorum":
        return (hq.EV_CHECK_QUORUM, 0, 0, 0, 0, 0, 0, 0, 0)
    if k == "campaign":
        return (hq.EV_ELECTION, 0, 0, 0, 0, 0, 0, 0, 0)
    if k == "propose":
        return (hq.EV_PROPOSE, 0, 0, 0, e[1], 0, 0, 0, 0)
    raise ValueError(k)


class OracleBackend:
    def __init__(self):
        from oracle import qref

        self.qref = qref
        self.groups = {}

    def add_group(self, cid, node, term, state, committed, last, term_start, members, log=None):
        """log: the node's log terms by index (StepGroup), None for the two-run history."""
        self.groups[cid] = self.qref.StepGroup(cid, node, term, state, committed, last,
                                               term_start, members, log)

    def step(self, per_group):
        out = {}
        for cid, events in per_group.items():
            check_phase_order(events)
            r = self.groups[cid].step(events)
            assert isinstance(r, dict), (cid, r, events)
            out[cid] = r
        return out

    def state(self, cid):
        return self.groups[cid].state()


class WorkerBackend:
    """stream=True: the step's events go in as an event stream (hq_events_encode ->
    hq_worker_step_stream) instead of rows."""

    def __init__(self, hq, n_max=8, seed=0, worker=None, on_device=False, stream=False):
        """stream: False (rows), True (stream with prefix arrays), "sized" (size words),
        "sized-column" (size words in, commits as a column out: HQ_WORKER_COMMIT_COLUMN),
        "sized-advance" (commits as 4-byte advances: HQ_WORKER_COMMIT_ADVANCE), "sized16" (2-byte
        size words, bytes only) or "sized16-slots" (2-byte words and the stream in pinned memory:
        the jobs path, commits as advances, ReadyToReads compact and in per-tile slots,
        HQ_WORKER_READY_SLOTS)."""
        self.hq = hq
        self.stream = stream
        slots = stream == "sized16-slots"
        self.w = worker if worker is not None else hq.Worker(
            0, n_max, on_device=on_device, commit_column=stream == "sized-column",
            commit_advance=stream in ("sized-advance", "sized16-slots"), ready_compact=slots,
            ready_slots=slots)
        self.pin = hq.Context(0) if slots else None
        self.pinned = {}
        self.rng = np.random.default_rng(seed)
        self.cids = []
        self.last_passes = 0
        self.last_decisions = 0

    def close(self):
        self.w.close()
        if self.pin:
            self.pin.close()

    def _pinned(self, key, a):
        """a copied into a pinned buffer kept for the next steps (grown when too small)."""
        buf = self.pinned.get(key)
        if buf is None or len(buf) < len(a):
            buf = self.pinned[key] = self.pin.pinned(max(len(a), 1) * 2, a.dtype)
        buf[:len(a)] = a
        return buf[:len(a)]

    def _sized(self, grp, sizes, n_events, data):
        """The SizedStream of this backend's form (4-byte words -> 2-byte ones, pinned)."""
        if str(self.stream).startswith("sized16"):
            sizes = self.hq.sizes16_of(sizes)
        if self.pin:
            sizes, data = self._pinned("sizes", sizes), self._pinned("data", data)
        return self.hq.SizedStream(grp, sizes, n_events, data)

    def add_group(self, cid, node, term, state, committed, last, term_start, members, log=None):
        # the worker holds term_start only: its term check is term_start <= q <= last, exact
        # because the leader's entries from its no-op on carry its term and earlier ones a lower
        # one (raft.go:911-922, entryutils.go:44-47); the oracle checks the whole history
        self.w.add_group(cid, node, term, state, committed, last, term_start, members)
        self.cids.append(cid)

    def build_inputs(self, per_group):
        """hq_worker_step input: the groups (in a random order) with their event lists.
        Returns ((handles, offsets, events), refs) with refs[event index] = (cid, pos)."""
        hq = self.hq
        cids = list(per_group)
        self.rng.shuffle(cids)
        handles, offsets, recs, refs = [], [0], [], {}
        for cid in cids:
            events = per_group[cid]
            check_phase_order(events)
            handles.append(self.w.find(cid))
            for pos, e in enumerate(events):
                refs[len(recs)] = (cid, pos)
                recs.append(event_record(hq, e))
            offsets.append(len(recs))
        self.last_cids = cids
        grp, off = np.array(handles, np.uint32), np.array(offsets, np.uint64)
        ev = np.array(recs, hq.EVENT_DTYPE)
        if str(self.stream).startswith("sized"):
            data, sizes = hq.encode_events_sized(off, ev)
            return self._sized(grp, sizes, len(ev), data), refs
        if self.stream:
            data, boff = hq.encode_events(off, ev)
            return (grp, off, boff, data), refs
        return (grp, off, ev), refs

    def step(self, per_group):
        arrs, refs = self.build_inputs(per_group)
        prev = {}                       # the committed indexes the advances add to
        if self.stream in ("sized-advance", "sized16-slots"):
            prev = {cid: int(self.w.get_group(cid)[0]["committed"]) for cid in self.last_cids}
        if isinstance(arrs, self.hq.SizedStream):
            res = self.w.step_sized(*arrs)
        else:
            res = self.w.step(*arrs) if len(arrs) == 3 else self.w.step_stream(*arrs)
        self.last_passes, self.last_decisions = res["gpu_passes"], res["decisions"]
        self.last_raw = res
        out = {cid: {"ready": [], "resps": [], "states": [], "dropped": [], "deferred": [],
                     "commit_changed": False} for cid in per_group}
        ready = res["ready"]
        if "ready_compact" in res or "ready_slots" in res:
            # the compact list and the slots, merged in list order (the reference's)
            lc = np.array(self.last_cids, np.uint64)
            ready = self.hq.merge_ready(res, lc, np.array([prev[c] for c in self.last_cids],
                                                          np.uint64))
        for r in ready:
            out[int(r["cluster_id"])]["ready"].append(
                (int(r["index"]), int(r["ctx_low"]), int(r["ctx_high"])))
        for r in res["read_resps"]:
            out[int(r["cluster_id"])]["resps"].append(
                (int(r["to"]), int(r["log_index"]), int(r["hint"]), int(r["hint_high"])))
        for r in res["state_changes"]:
            out[int(r["cluster_id"])]["states"].append(
                (int(r["term"]), int(r["state"]), int(r["reason"])))
        for r in res["dropped_reads"]:
            out[int(r["cluster_id"])]["dropped"].append(
                (int(r["ctx_low"]), int(r["ctx_high"]), int(r["from"]), int(r["reason"])))
        for r in res["deferred"]:
            cid, pos = refs[int(r)]
            out[cid]["deferred"].append(pos)
        for cid in out:
            out[cid]["deferred"].sort()
        for r in res["commits"]:
            out[int(r["cluster_id"])]["commit_changed"] = True
        col = res.get("committed_column")
        if col is not None:             # one word per listed group, in input order
            assert len(col) == len(self.last_cids) and res["n_commits"] == int((col != 0).sum())
            for cid, v in zip(self.last_cids, col.tolist()):
                if v:
                    out[cid]["commit_changed"] = True
                    out[cid]["_col"] = v
        adv = res.get("committed_advance")
        if adv is not None:             # one advance per listed group, in input order
            assert len(adv) == len(self.last_cids) and res["n_commits"] == int((adv != 0).sum())
            for cid, v in zip(self.last_cids, adv.tolist()):
                if v:
                    out[cid]["commit_changed"] = True
                    out[cid]["_col"] = prev[cid] + v
        for cid in out:
            out[cid]["committed"] = int(self.w.get_group(cid)[0]["committed"])
            assert out[cid].pop("_col", out[cid]["committed"]) == out[cid]["committed"]
        out["_fallback"] = [int(x) for x in res["fallback_groups"]]
        return out

    def state(self, cid):
        g, m, r = self.w.get_group(cid)
        members = [(int(x["node_id"]), int(x["match"]), int(x["role"]), int(x["active"]))
                   for x in m]
        reads = [(int(x["index"]), int(x["from"]), (int(x["ctx_low"]), int(x["ctx_high"])),
                  int(x["n_confirmed"])) for x in r]
        return (int(g["term"]), int(g["state"]), int(g["committed"]), int(g["last_index"]),
                int(g["term_start"]), members, reads)


def same_step(oracle_out, worker_out, cid):
    """Per-group step results must be identical."""
    o, w = oracle_out[cid], worker_out[cid]
    for k in ("committed", "commit_changed", "ready", "resps", "states", "dropped", "deferred"):
        assert o[k] == w[k], (cid, k, o[k], w[k])


class WireBackend(WorkerBackend):
    """The step worker fed from the wire: every received message of the step is marshalled into
    raftpb.MessageBatch bytes (tests/wire_encode.py, the gogo layout), the clusters' queues
    interleaved in arrival order and cut into several batches, plus batches and messages the
    reference drops before Peer.Handle (a foreign deployment id, SnapshotReceived, a cluster this
    host does not run); hq_wire decodes them and assembles the step input (local events via
    hq_wire_add_local). Results must equal the event-row path's."""

    DEPLOYMENT = 0x5EED

    def __init__(self, hq, n_max=8, seed=0, worker=None, on_device=False, stream=False):
        super().__init__(hq, n_max, seed, worker, on_device, stream)
        self.wire = hq.Wire(self.DEPLOYMENT)
        self.last_stats = None
        # "sized16-slots": the production feed — the wire attached to the worker, the step in
        # handle order straight into pinned stream buffers (hq_wire_step_sized)
        self.attached = stream == "sized16-slots"
        if self.attached:
            self.wire.attach(self.w)

    def close(self):
        self.wire.close()
        super().close()

    def build_inputs(self, per_group):
        import wire_encode as we

        hq, rng, wire = self.hq, self.rng, self.wire
        wire.reset()
        cids = list(per_group)
        rng.shuffle(cids)
        queues = {}
        for cid in cids:
            events = per_group[cid]
            check_phase_order(events)
            local = [event_record(hq, e) for e in events if e[0] != "msg"]
            if local:
                wire.add_local(cid, np.array(local, hq.EVENT_DTYPE))
            queues[cid] = [we.message(type=e[1], to=1, frm=e[2], cluster_id=cid, term=e[3],
                                      log_index=e[4], hint=e[5], hint_high=e[6],
                                      reject=bool(e[7]))
                           for e in events if e[0] == "msg"]
        # arrival order: a random merge of the clusters' queues (each kept in order), with
        # messages the reference drops before the queue mixed in
        stream, heads = [], {c: 0 for c in cids}
        live = [c for c in cids if queues[c]]
        while live:
            c = live[int(rng.integers(len(live)))]
            stream.append(queues[c][heads[c]])
            heads[c] += 1
            if heads[c] == len(queues[c]):
                live.remove(c)
            r = rng.random()
            if r < 0.02:   # SnapshotReceived: handled aside (nodehost.go:2039-2044)
                stream.append(we.message(type=22, frm=2, cluster_id=c))
            elif r < 0.04:  # a cluster this worker does not run: dropped (nodehost.go:2045)
                stream.append(we.message(type=13, frm=2, cluster_id=(1 << 62) + c, term=1,
                                         log_index=5))
        cut = sorted(set(int(x) for x in rng.integers(0, len(stream) + 1, 3)))
        parts = [stream[a:b] for a, b in zip([0] + cut, cut + [len(stream)])]
        for i, p in enumerate(parts):
            wire.add_batch(we.batch(p, deployment_id=self.DEPLOYMENT, source_address=b"n2:1"))
            if i == 0:   # a foreign deployment's batch: dropped whole (transport.go:291-295)
                wire.add_batch(we.batch(p, deployment_id=self.DEPLOYMENT + 1))
                if p:    # a truncated batch: rejected, none of its messages queued
                    b = we.batch(p, deployment_id=self.DEPLOYMENT, source_address=b"n2:1")
                    tail = len(we.batch([], deployment_id=self.DEPLOYMENT, source_address=b"n2:1"))
                    try:       # (the last message one byte short of its length)
                        wire.add_batch(b[:len(b) - tail - 1])
                    except hq.HQError:
                        pass
                    else:
                        raise AssertionError("a truncated MessageBatch was accepted")
        if self.attached:
            # every handle in order (a group without events has size 0); handles are the order
            # the groups were added in
            ne = sum(len(v) for v in per_group.values())
            data = self._pinned("wdata", np.zeros(ne * hq.HQ_EVENT_STREAM_MAX + 64, np.uint8))
            sizes = self._pinned("wsizes", np.zeros(len(self.cids), np.uint16))
            ss, st = wire.step_sized(data, sizes)
            self.last_stats = st
            refs, k = {}, 0
            for cid in self.cids:
                for pos in range(len(per_group.get(cid, ()))):
                    refs[k] = (cid, pos)
                    k += 1
            assert k == ss[2] and len(ss[1]) == len(self.cids)
            self.last_cids = list(self.cids)
            return ss, refs
        if self.stream:                       # hq_wire_step_stream
            grp, off, boff, data, st = wire.step_stream(self.w)
        else:
            grp, off, ev, st = wire.step_input(self.w)
        self.last_stats = st
        # event index -> (cluster, position in its per_group list): the assembled rows keep
        # node.handleEvents order, as the per_group lists do
        refs = {}
        handle_cid = {self.w.find(c): c for c in cids}
        for i, h in enumerate(grp):
            cid = handle_cid[int(h)]
            for pos, k in enumerate(range(int(off[i]), int(off[i + 1]))):
                refs[k] = (cid, pos)
            assert int(off[i + 1]) - int(off[i]) == len(per_group[cid])
        assert sorted(handle_cid[int(h)] for h in grp) == sorted(c for c in cids
                                                                 if per_group[c])
        self.last_cids = [handle_cid[int(h)] for h in grp]
        if str(self.stream).startswith("sized"):
            sizes = (np.diff(off) | (np.diff(boff) << np.uint64(16))).astype(np.uint32)
            return self._sized(grp, sizes, int(off[-1]), data), refs
        return ((grp, off, boff, data) if self.stream else (grp, off, ev)), refs
