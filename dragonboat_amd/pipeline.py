"""Host-fed steps into the device-resident progress table, pipelined over
several contexts.

A step worker that keeps its leader groups' quorum state on the GPU feeds each step as two
pinned host arrays and reads back the decisions:

  * leader appends (``hq_append_update`` pairs: group, new lastIndex) — ``appendEntries``'
    lastIndex / self-match / current-term bits (raft.go:912-922);
  * follower match deltas (``hq_match_update`` pairs: group << 8 | slot, index) —
    ``remote.tryUpdate`` per accepted ReplicateResp (remote.go:123-133, raft.go:1671-1700);
  * then ``tryCommit`` over every group in place (mask form), and a readback of the changed
    bitmap and the committed column (``commitTo`` results, logentry.go:323-332).

With ``depth`` = 1 every step runs on one stream: the next step's host-to-device copies wait for
the previous readback. With ``depth`` = 2 the steps alternate between two contexts; each step's
kernels are ordered after the previous step (``hq_wait_for``), so the decisions are those of the
serial run, while its copies overlap the previous step's kernels and readback (the copy engines
run beside the compute queues; PCIe is full duplex). Every decision is a kernel of
libhipquorum.so; nothing here computes.
"""
from __future__ import annotations

import numpy as np

from . import hipquorum as hq


class HostFedPipeline:
    def __init__(self, device: int, G: int, n: int, max_appends: int, max_updates: int,
                 depth: int = 2, ring_len: int = 16, compact: bool = False):
        """compact: 8-byte records (hq_append_count_dev: group << 32 | entries;
        hq_ingest_lag_dev: group << 32 | slot << 28 | lastIndex - index) instead of the 16-byte
        hq_append_update / hq_match_update pairs — half the PCIe bytes per step."""
        if depth < 1:
            raise ValueError("depth must be >= 1")
        self.G, self.n, self.R, self.depth = G, n, ring_len, depth
        self.compact = compact
        w = 1 if compact else 2     # uint64 words per record
        self.ctxs = [hq.Context(device) for _ in range(depth)]
        c0 = self.ctxs[0]
        self.table = hq.alloc_commit(c0, G, n, hq.HQ_FORM_TERM_MASK, ring_len)
        a = self.table.args()
        a.committed_out = a.committed_in      # decided in place
        self.args = a
        self.max_appends, self.max_updates = max_appends, max_updates
        # per context: device staging for the step's inputs, pinned buffers for its results
        self.dapp = [c.empty(w * max(1, max_appends), np.uint64) for c in self.ctxs]
        self.dupd = [c.empty(w * max(1, max_updates), np.uint64) for c in self.ctxs]
        self.out_chg = [c.pinned(hq.words64(G), np.uint64) for c in self.ctxs]
        self.out_com = [c.pinned(G, np.uint64) for c in self.ctxs]
        self._last = None

    # -- setup ----------------------------------------------------------------------------
    def synth(self, spec: hq.SynthSpec) -> None:
        """Initial table from the device generator (DESIGN.md "Synthetic inputs")."""
        self.ctxs[0].synth_commit_dev(spec, self.table.args())
        self.ctxs[0].sync()

    def upload(self, match, committed, last_index, term_mask) -> None:
        c = self.ctxs[0]
        for dst, src in ((self.table.match, match), (self.table.committed_in, committed),
                         (self.table.last_index, last_index), (self.table.term_mask, term_mask)):
            c.h2d_async(dst, np.ascontiguousarray(src, dst.dtype))
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
        x = self.ctxs[k]
        if n_appends:
            x.h2d_async(self.dapp[k], appends[:w * n_appends])
        if n_updates:
            x.h2d_async(self.dupd[k], updates[:w * n_updates])
        if self._last is not None and self._last is not x:
            x.wait_for(self._last)        # kernels after the previous step (and its readback)
        t = self.table
        if self.compact:
            if n_appends:
                x.append_count_dev(self.dapp[k], n_appends, t.last_index, t.match, t.term_mask,
                                   self.R, self.G)
            if n_updates:
                x.ingest_lag_dev(self.dupd[k], n_updates, t.match, self.G, t.last_index, self.G,
                                 self.n)
        else:
            if n_appends:
                x.append_dev(self.dapp[k], n_appends, t.last_index, t.match, t.term_mask,
                             self.R, self.G)
            if n_updates:
                x.ingest_match_dev(self.dupd[k], n_updates, t.match, self.G, self.G, self.n)
        x.commit_dev(self.args)
        x.d2h_async(self.out_chg[k], t.changed)
        x.d2h_async(self.out_com[k], t.committed_in)
        self._last = x
        return k

    def results(self, k: int):
        """(changed bitmap, committed column) of the last step that used result buffers k."""
        self.ctxs[k].sync()
        return self.out_chg[k], self.out_com[k]

    def sync(self) -> None:
        for c in self.ctxs:
            c.sync()

    def close(self) -> None:
        for c in self.ctxs[1:]:
            c.close()
        self.ctxs[0].close()   # owns the table
