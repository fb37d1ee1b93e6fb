"""Host-fed steps into the device-resident progress table, pipelined over
several contexts.

The table is the headline kernel's own input: HQ_LAYOUT_TILES_LEADER tiles (match slots 1..n-1,
committed, lastIndex, term mask or term start per 128-group tile; the leader's match is its
lastIndex, raft.go:918), kept on the GPU across steps and decided in place by the headline kernel
(``k_commit_big<n, form, 2, false, 3>``, hq_commit_dev with HQ_LAYOUT_IN_PLACE). A step worker
feeds each step as two pinned host arrays and reads back the decisions:

  * leader appends (``hq_append_update`` pairs: group, new lastIndex; or 8-byte
    group << 32 | entries) — ``appendEntries``' lastIndex and current-term bits (raft.go:911-922);
  * follower match deltas (``hq_match_update`` pairs: group << 8 | slot, index; or 8-byte
    group << 32 | slot << 28 | lag below lastIndex) — ``remote.tryUpdate`` per accepted
    ReplicateResp (remote.go:123-133, raft.go:1671-1700);
  * then ``tryCommit`` over every group in place, and a readback of the changed bitmap, the
    fallback bitmap and the committed indexes (``commitTo`` results, logentry.go:323-332).

Fallback groups (mask form: lastIndex - committed > ring_len, or committed > lastIndex) are NOT
decided by the kernel: their committed index is left as it was and their bit is set in the
fallback bitmap that ``results`` returns. The caller decides them with the CPU tryCommit
(raft.go:888-909) and writes the new committed index back into the table (``set_committed``).

With ``depth`` = 1 every step runs on one stream: the next step's host-to-device copies wait for
the previous readback. With ``depth`` = 2 the steps alternate between two contexts; each step's
kernels are ordered after the previous step's kernels (``hq_wait_for``), so the decisions are
those of the serial run, while its copies overlap the previous step's kernels and readback (the
copy engines run beside the compute queues; PCIe is full duplex). The readback of a step runs on
a context of its own, from result buffers of its own (one set per pipeline slot), so the next
step's kernels need not wait for it: a slot's buffers are reused only after its readback of
``depth`` steps earlier has finished. ``grouped``: the caller's records of one
key are adjacent (node by node, as a step worker emits them), so the ingest kernels reduce runs
in registers and write without atomics (HQ_INGEST_GROUPED). Every decision is a kernel of
libhipquorum.so; nothing here computes.
"""
from __future__ import annotations

import numpy as np

from . import hipquorum as hq


class HostFedPipeline:
    def __init__(self, device: int, G: int, n: int, max_appends: int, max_updates: int,
                 depth: int = 2, ring_len: int = 16, compact: bool = False,
                 form: int = hq.HQ_FORM_TERM_MASK, grouped: bool = False,
                 zero_copy: bool = False):
        """compact: 8-byte records (hq_table_append_count_dev: group << 32 | entries;
        hq_table_ingest_lag_dev: group << 32 | slot << 28 | lastIndex - index) instead of the
        16-byte hq_append_update / hq_match_update pairs — half the PCIe bytes per step.
        zero_copy: no copies at all — the append / ingest kernels read the caller's pinned records
        over PCIe and the decision writes the changed / fallback bitmaps and the committed column
        straight into this slot's pinned result buffers (``depth`` result slots), every step on
        one stream: no copy engine and no cross-stream wait is involved. The records must then be
        pinned host (``Context.pinned``) or device memory (``step`` raises ValueError otherwise,
        instead of letting a kernel fault on pageable memory), and they must stay unmodified until
        that step's ``results`` / ``sync`` returns: the kernels read them asynchronously."""
        if depth < 1:
            raise ValueError("depth must be >= 1")
        self.zero_copy = zero_copy
        if form not in (hq.HQ_FORM_TERM_MASK, hq.HQ_FORM_TERM_START):
            raise ValueError("the table holds the term-mask or term-start form")
        self.G, self.n, self.R, self.depth, self.form = G, n, ring_len, depth, form
        self.compact = compact
        self.flags = hq.HQ_INGEST_GROUPED if grouped else 0
        w = 1 if compact else 2     # uint64 words per record
        # zero_copy: one stream (a second one for the committed column's extraction measured no
        # faster: the GPU's posted PCIe writes hold back the next step's record reads, which may
        # not pass them, profiles/r02k/)
        self.ctxs = [hq.Context(device) for _ in range(1 if zero_copy else depth)]
        c0 = self.ctxs[0]
        self.layout = hq.HQ_LAYOUT_TILES_LEADER
        self.tiles = c0.empty(hq.commit_tiles(G) * hq.commit_tile_words(n, form, self.layout),
                              np.uint64)
        # readback contexts (one stream per pipeline slot; the step's own with depth 1)
        self.rbs = [hq.Context(device) for _ in range(depth)] \
            if depth > 1 and not zero_copy else self.ctxs
        # per slot: the device result buffers the decision writes and the readback reads
        self.changed = [c0.empty(hq.words64(G), np.uint64) for _ in range(depth)]
        self.fallback = [c0.empty(hq.words64(G), np.uint64) for _ in range(depth)]
        self.committed = [c0.empty(G, np.uint64) for _ in range(depth)]
        self.args = []
        for k in range(depth):
            a = hq.CommitArgs()
            a.G, a.n_max, a.form, a.ring_len = G, n, form, ring_len
            a.layout = hq.HQ_LAYOUT_TILES_LEADER | hq.HQ_LAYOUT_IN_PLACE
            a.match, a.changed, a.fallback = (self.tiles.ptr, self.changed[k].ptr,
                                              self.fallback[k].ptr)
            self.args.append(a)
        self.max_appends, self.max_updates = max_appends, max_updates
        # per context: device staging for the step's inputs; per slot: pinned result buffers
        self.dapp = [c.empty(w * max(1, max_appends), np.uint64) for c in self.ctxs]
        self.dupd = [c.empty(w * max(1, max_updates), np.uint64) for c in self.ctxs]
        self.out_chg = [c0.pinned(hq.words64(G), np.uint64) for _ in range(depth)]
        self.out_fb = [c0.pinned(hq.words64(G), np.uint64) for _ in range(depth)]
        self.out_com = [c0.pinned(G, np.uint64) for _ in range(depth)]
        if zero_copy:   # the decision writes the results where the caller reads them
            for k, a in enumerate(self.args):
                a.changed = self.out_chg[k].ctypes.data
                a.fallback = self.out_fb[k].ctypes.data
        self._last = None

    # -- setup ----------------------------------------------------------------------------
    def synth(self, spec: hq.SynthSpec) -> None:
        """Initial table from the device generator (DESIGN.md "Synthetic inputs"), cut into the
        leader-row tiles on the device (the generator's slot 0 is lastIndex)."""
        c = self.ctxs[0]
        b = hq.alloc_commit(c, self.G, self.n, self.form, self.R)
        c.synth_commit_dev(spec, b.args())
        c.tile_commit_dev(b.args(), self.tiles, self.layout)
        c.sync()
        hq.free_commit(c, b)

    def upload(self, match, committed, last_index, aux) -> None:
        """Initial table from host columns (match slot-major [n][G], slot 0 = lastIndex; aux =
        the u16 term mask or the u64 term_start). The host packer refuses a group whose slot 0
        is not its lastIndex."""
        G, n = self.G, self.n
        cols = [np.ascontiguousarray(x, t) for x, t in
                ((match, np.uint64), (committed, np.uint64), (last_index, np.uint64))]
        aux = np.ascontiguousarray(aux, np.uint16 if self.form == hq.HQ_FORM_TERM_MASK
                                   else np.uint64)
        a = hq.CommitArgs()
        a.G, a.n_max, a.form, a.ring_len, a.match_stride = G, n, self.form, self.R, G
        a.match, a.committed_in, a.last_index = (x.ctypes.data for x in cols)
        if self.form == hq.HQ_FORM_TERM_MASK:
            a.term_mask = aux.ctypes.data
        else:
            a.term_start = aux.ctypes.data
        tiles = hq.tile_commit_host(a, self.layout)
        c = self.ctxs[0]
        c.h2d_async(self.tiles, tiles)
        c.sync()

    def set_committed(self, groups, committed) -> None:
        """Write committed indexes decided on the CPU (the fallback groups) into the table."""
        c = self.ctxs[0]
        self.sync()
        tiles = c.download(self.tiles)
        hq.tile_view(tiles, self.G, self.n, self.form, self.layout).set_row(
            "committed", np.asarray(groups, np.int64), np.asarray(committed, np.uint64))
        c.h2d_async(self.tiles, tiles)
        c.sync()

    # -- steps ----------------------------------------------------------------------------
    def step(self, i: int, appends: np.ndarray, n_appends: int, updates: np.ndarray,
             n_updates: int) -> int:
        """Enqueue step i (asynchronous). appends / updates: flat pinned uint64 arrays of
        (group, new_last) and (group << 8 | slot, index) pairs, or in the compact form one word
        each (``hipquorum.pack_append_counts`` / ``pack_lag_updates``; lags relative to lastIndex
        after this step's appends). Returns the index of the result buffers the step reads back
        into (``results``)."""
        if n_appends > self.max_appends or n_updates > self.max_updates:
            raise ValueError("step larger than the staging buffers")
        w = 1 if self.compact else 2
        k = i % self.depth
        G, n, f = self.G, self.n, self.form
        if self.zero_copy:
            x = self.ctxs[0]
            app, upd = appends[:w * n_appends], updates[:w * n_updates]
            for name, arr, cnt in (("appends", app, n_appends), ("updates", upd, n_updates)):
                if cnt and hq.pointer_kind(arr) == hq.HQ_PTR_UNREGISTERED:
                    raise ValueError(f"zero_copy: {name} must be pinned host or device memory "
                                     "(Context.pinned), not pageable host memory")
            if self.compact:
                if n_appends:
                    x.table_append_count_dev(app, n_appends, self.tiles, G, n, f, self.R,
                                             self.flags)
                if n_updates:
                    x.table_ingest_lag_dev(upd, n_updates, self.tiles, G, n, f, self.flags)
            else:
                if n_appends:
                    x.table_append_dev(app, n_appends, self.tiles, G, n, f, self.R, self.flags)
                if n_updates:
                    x.table_ingest_match_dev(upd, n_updates, self.tiles, G, n, f, self.flags)
            x.commit_dev(self.args[k])
            x.table_committed_dev(self.tiles, G, n, f, self.out_com[k])
            self._last = x
            return k
        x = self.ctxs[k]
        if n_appends:
            x.h2d_async(self.dapp[k], appends[:w * n_appends])
        if n_updates:
            x.h2d_async(self.dupd[k], updates[:w * n_updates])
        rb = self.rbs[k]
        if self._last is not None and self._last is not x:
            x.wait_for(self._last)        # kernels after the previous step's kernels
        if rb is not x:
            x.wait_for(rb)                # slot k's result buffers read back (step i - depth)
        if self.compact:
            if n_appends:
                x.table_append_count_dev(self.dapp[k], n_appends, self.tiles, G, n, f, self.R,
                                         self.flags)
            if n_updates:
                x.table_ingest_lag_dev(self.dupd[k], n_updates, self.tiles, G, n, f, self.flags)
        else:
            if n_appends:
                x.table_append_dev(self.dapp[k], n_appends, self.tiles, G, n, f, self.R,
                                   self.flags)
            if n_updates:
                x.table_ingest_match_dev(self.dupd[k], n_updates, self.tiles, G, n, f,
                                         self.flags)
        x.commit_dev(self.args[k])
        x.table_committed_dev(self.tiles, G, n, f, self.committed[k])
        if rb is not x:
            rb.wait_for(x)                # the readback after this step's kernels
        rb.d2h_async(self.out_chg[k], self.changed[k])
        rb.d2h_async(self.out_fb[k], self.fallback[k])
        rb.d2h_async(self.out_com[k], self.committed[k])
        self._last = x
        return k

    def results(self, k: int):
        """(changed bitmap, committed column, fallback bitmap) of the last step that used
        result buffers k. Groups with a fallback bit were not decided (their committed index is
        the previous one): decide them on the CPU and write them back with set_committed."""
        if self.zero_copy:
            self.sync()
        else:
            self.rbs[k].sync()
        return self.out_chg[k], self.out_com[k], self.out_fb[k]

    def sync(self) -> None:
        for c in self.ctxs + (self.rbs if self.rbs is not self.ctxs else []):
            c.sync()

    def close(self) -> None:
        self.sync()
        if self.rbs is not self.ctxs:
            for c in self.rbs:
                c.close()
        for c in self.ctxs[1:]:
            c.close()
        self.ctxs[0].close()   # owns the table
