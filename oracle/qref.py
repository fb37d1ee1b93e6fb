"""ctypes binding of the CPU oracle (oracle/build/libqref.so). TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import this module, and only
as the checker or the timed CPU baseline — never as part of the product path.
Parity status: pinned by the reference's own known-answer tables (tests/golden/), see qref.h.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "build", "libqref.so")

QREF_FOLLOWER, QREF_CANDIDATE, QREF_LEADER = 0, 1, 2
QREF_PANIC = -100
QREF_MAX_NODES = 16
QREF_MAX_PENDING = 64

_vp = ctypes.c_void_p
_u64 = ctypes.c_uint64


class QrefCommitArgs(ctypes.Structure):
    _fields_ = [
        ("G", _u64), ("n_max", ctypes.c_uint32), ("form", ctypes.c_uint32),
        ("ring_len", ctypes.c_uint32), ("reserved", ctypes.c_uint32), ("match_stride", _u64),
        ("match", _vp), ("n_voting", _vp), ("committed_in", _vp), ("committed_out", _vp),
        ("last_index", _vp), ("term_start", _vp), ("term", _vp), ("ring", _vp),
        ("changed", _vp), ("fallback", _vp), ("term_mask", _vp),
    ]


class QgenSpec(ctypes.Structure):
    _fields_ = [
        ("seed", _u64), ("G", _u64), ("cid_base", _u64), ("cid_stride", _u64),
        ("n_max", ctypes.c_uint32), ("mixed_n", ctypes.c_uint32),
        ("ring_len", ctypes.c_uint32), ("parity_extras", ctypes.c_uint32),
    ]


class SysCtx(ctypes.Structure):
    _fields_ = [("low", _u64), ("high", _u64)]


class ReadStatus(ctypes.Structure):
    _fields_ = [("index", _u64), ("from_", _u64), ("ctx", SysCtx), ("n_confirmed", ctypes.c_int),
                ("confirmed", _u64 * QREF_MAX_NODES)]


class ReadIndex(ctypes.Structure):
    _fields_ = [("pending", ReadStatus * QREF_MAX_PENDING), ("n_pending", ctypes.c_int),
                ("queue", SysCtx * QREF_MAX_PENDING), ("n_queue", ctypes.c_int)]


class Votes(ctypes.Structure):
    _fields_ = [("n", ctypes.c_int), ("from_", _u64 * QREF_MAX_NODES),
                ("granted", ctypes.c_int * QREF_MAX_NODES)]


QREF_STEP_MAX_MEMBERS = 16
QREF_LOG_MAX_RUNS = 64
QREF_STEP_MAX_OUT = 64
EV_READ, EV_MSG, EV_CHECK_QUORUM, EV_CAMPAIGN, EV_PROPOSE = 1, 2, 3, 4, 5


class Member(ctypes.Structure):
    _fields_ = [("node_id", _u64), ("match", _u64), ("role", ctypes.c_uint32),
                ("active", ctypes.c_uint32)]


class Event(ctypes.Structure):
    _fields_ = [("kind", ctypes.c_uint32), ("type", ctypes.c_uint32), ("from_", _u64),
                ("term", _u64), ("log_index", _u64), ("hint", _u64), ("hint_high", _u64),
                ("reject", ctypes.c_uint32), ("reserved", ctypes.c_uint32)]


class Group(ctypes.Structure):
    _fields_ = [("cluster_id", _u64), ("node_id", _u64), ("term", _u64), ("state", ctypes.c_int),
                ("n_members", ctypes.c_int), ("committed", _u64), ("last", _u64),
                ("term_start", _u64), ("members", Member * QREF_STEP_MAX_MEMBERS),
                ("ri", ctypes.POINTER(ReadIndex)), ("votes", Votes),
                ("first_minus_1", _u64), ("n_runs", ctypes.c_int),
                ("run_start", _u64 * QREF_LOG_MAX_RUNS), ("run_term", _u64 * QREF_LOG_MAX_RUNS)]


class _Ready(ctypes.Structure):
    _fields_ = [("index", _u64), ("low", _u64), ("high", _u64)]


class _Resp(ctypes.Structure):
    _fields_ = [("to", _u64), ("index", _u64), ("hint", _u64), ("hint_high", _u64)]


class _State(ctypes.Structure):
    _fields_ = [("term", _u64), ("state", ctypes.c_uint32), ("reason", ctypes.c_uint32)]


class _Dropped(ctypes.Structure):
    _fields_ = [("low", _u64), ("high", _u64), ("from_", _u64), ("reason", ctypes.c_uint32),
                ("reserved", ctypes.c_uint32)]


class StepOut(ctypes.Structure):
    _fields_ = [("committed", _u64), ("commit_changed", ctypes.c_int), ("n_ready", ctypes.c_int),
                ("n_resps", ctypes.c_int), ("n_states", ctypes.c_int), ("n_dropped", ctypes.c_int),
                ("n_deferred", ctypes.c_int), ("ready", _Ready * QREF_STEP_MAX_OUT),
                ("resps", _Resp * QREF_STEP_MAX_OUT), ("states", _State * QREF_STEP_MAX_OUT),
                ("dropped", _Dropped * QREF_STEP_MAX_OUT),
                ("deferred", ctypes.c_uint32 * QREF_STEP_MAX_OUT)]


TERM_FN = ctypes.CFUNCTYPE(_u64, _vp, _u64)


class QrefLog(ctypes.Structure):
    _fields_ = [("first_minus_1", _u64), ("last", _u64), ("committed", _u64),
                ("term_at", TERM_FN), ("ud", _vp)]


def build() -> None:
    subprocess.run(["make", "-s", "-C", _HERE], check=True)


def load() -> ctypes.CDLL:
    if not os.path.exists(LIB_PATH):
        build()
    lib = ctypes.CDLL(LIB_PATH)
    sig = {
        "qref_num_voting_members": (ctypes.c_int, [ctypes.c_int, ctypes.c_int]),
        "qref_quorum": (ctypes.c_int, [ctypes.c_int]),
        "qref_is_single_node_quorum": (ctypes.c_int, [ctypes.c_int]),
        "qref_sort_match_values": (None, [_vp, ctypes.c_int]),
        "qref_log_term": (_u64, [ctypes.POINTER(QrefLog), _u64]),
        "qref_log_try_commit": (ctypes.c_int, [ctypes.POINTER(QrefLog), _u64, _u64]),
        "qref_try_commit": (ctypes.c_int, [_vp, ctypes.c_int, _vp, ctypes.c_int,
                                           ctypes.POINTER(QrefLog), _u64, _vp]),
        "qref_quorum_match_by_count": (_u64, [_vp, ctypes.c_int]),
        "qref_ri_init": (None, [ctypes.POINTER(ReadIndex)]),
        "qref_ri_add_request": (ctypes.c_int, [ctypes.POINTER(ReadIndex), _u64, SysCtx, _u64]),
        "qref_ri_has_pending": (ctypes.c_int, [ctypes.POINTER(ReadIndex)]),
        "qref_ri_confirm": (ctypes.c_int, [ctypes.POINTER(ReadIndex), SysCtx, _u64, ctypes.c_int,
                                           ctypes.POINTER(ReadStatus)]),
        "qref_votes_reset": (None, [ctypes.POINTER(Votes)]),
        "qref_handle_vote_resp": (ctypes.c_int, [ctypes.POINTER(Votes), _u64, ctypes.c_int]),
        "qref_candidate_vote_resp": (ctypes.c_int, [ctypes.POINTER(Votes), _u64, ctypes.c_int,
                                                    ctypes.c_int, ctypes.c_int]),
        "qref_leader_has_quorum": (ctypes.c_int, [_vp, _vp, ctypes.c_int, _u64]),
        "qref_commit_batch": (ctypes.c_int, [ctypes.POINTER(QrefCommitArgs), ctypes.c_int]),
        "qref_readindex_batch": (ctypes.c_int, [_u64, _vp, _vp, ctypes.c_uint32, _vp, _vp,
                                                ctypes.c_int]),
        "qref_vote_batch": (ctypes.c_int, [_u64, _vp, _vp, _vp, ctypes.c_uint32, _vp, _vp,
                                           ctypes.c_int]),
        "qref_check_quorum_batch": (ctypes.c_int, [_u64, _vp, _vp, ctypes.c_uint32,
                                                   ctypes.c_uint32, _vp, _vp, ctypes.c_int]),
        "qgen_splitmix64": (_u64, [ctypes.POINTER(_u64)]),
        "qgen_commit": (ctypes.c_int, [ctypes.POINTER(QgenSpec), ctypes.POINTER(QrefCommitArgs)]),
        "qgen_bitmaps": (ctypes.c_int, [ctypes.POINTER(QgenSpec), _vp, _vp, _vp, _vp]),
        "qref_fnv1a64": (_u64, [_vp, ctypes.c_size_t]),
        "qref_readindex_multi_batch": (ctypes.c_int, [_u64, ctypes.c_uint32, ctypes.c_uint32, _vp,
                                                      _vp, _vp, _vp, ctypes.c_uint32, _vp, _vp,
                                                      _vp, _vp, ctypes.c_int]),
        "qgen_c1_stream": (ctypes.c_int, [_u64, _u64, _u64, _u64, _vp, _vp]),
        "qref_group_init": (ctypes.c_int, [_vp, _u64, _u64, _u64, ctypes.c_int, _u64, _u64, _u64,
                                           _vp, ctypes.c_int]),
        "qref_group_step": (ctypes.c_int, [_vp, _vp, ctypes.c_int, _vp]),
        "qref_group_set_log": (ctypes.c_int, [_vp, _u64, ctypes.c_int, _vp, _vp]),
        "qref_group_free": (None, [_vp]),
        "qref_groups_new": (_vp, [_u64]),
        "qref_groups_free": (None, [_vp, _u64]),
        "qref_groups_init": (ctypes.c_int, [_vp, _u64, _vp, _vp]),
        "qref_step_batch": (ctypes.c_int, [_vp, _u64, _u64, _vp, _vp, _vp, ctypes.c_int, _vp]),
        "qref_digest_ready_term": (_u64, [_u64, _u64, _u64, _u64]),
        "qref_digest_commit_term": (_u64, [_u64, _u64]),
        "qref_c1_run": (ctypes.c_int, [_u64, _vp, _vp, _u64, _u64, _vp]),
        "qref_ingest_match": (_u64, [_vp, _u64, _vp, _u64, _u64, ctypes.c_uint32]),
        "qref_ingest_ack": (_u64, [_vp, _u64, _vp, _u64, ctypes.c_uint32]),
        "qref_append": (_u64, [_vp, _u64, _vp, _vp, _vp, ctypes.c_uint32, _u64]),
    }
    for name, (res, args) in sig.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    return lib


lib = load()


def _ptr(a):
    return None if a is None else a.ctypes.data_as(_vp)


# ------------------------------------------------------------------------ scalar helpers ----
def quorum(n: int) -> int:
    return lib.qref_quorum(n)


def sort_match_values(vals):
    a = np.array(vals, dtype=np.uint64)
    lib.qref_sort_match_values(_ptr(a), len(a))
    return [int(x) for x in a]


class EntryLog:
    """A log view: ``terms`` maps index -> term for indexes in [first_minus_1, last]."""

    def __init__(self, first_minus_1: int, last: int, committed: int, terms: dict[int, int]):
        self._terms = dict(terms)
        self._fn = TERM_FN(lambda ud, i: self._terms.get(int(i), 0))
        self.c = QrefLog(first_minus_1, last, committed, self._fn, None)

    @property
    def committed(self) -> int:
        return int(self.c.committed)

    def term(self, index: int) -> int:
        return int(lib.qref_log_term(ctypes.byref(self.c), index))


def try_commit(remote_match, witness_match, log: EntryLog, term: int) -> tuple[int, int]:
    """raft.tryCommit; returns (rc, q)."""
    r = np.array(remote_match, dtype=np.uint64)
    w = np.array(witness_match, dtype=np.uint64)
    q = _u64(0)
    rc = lib.qref_try_commit(_ptr(r), len(r), _ptr(w) if len(w) else None, len(w),
                             ctypes.byref(log.c), term, ctypes.byref(q))
    return rc, int(q.value)


class PyReadIndex:
    def __init__(self):
        self.c = ReadIndex()
        lib.qref_ri_init(ctypes.byref(self.c))
        self._out = (ReadStatus * QREF_MAX_PENDING)()

    def add_request(self, index: int, ctx: tuple[int, int], frm: int) -> int:
        return lib.qref_ri_add_request(ctypes.byref(self.c), index, SysCtx(*ctx), frm)

    def confirm(self, ctx: tuple[int, int], frm: int, q: int):
        rc = lib.qref_ri_confirm(ctypes.byref(self.c), SysCtx(*ctx), frm, q, self._out)
        if rc == QREF_PANIC:
            return "panic"
        if rc == 0:
            return None
        return [(int(s.index), int(s.from_), (int(s.ctx.low), int(s.ctx.high)))
                for s in self._out[:rc]]

    @property
    def n_pending(self):
        return self.c.n_pending

    @property
    def n_queue(self):
        return self.c.n_queue


class PyVotes:
    def __init__(self):
        self.c = Votes()
        lib.qref_votes_reset(ctypes.byref(self.c))

    def handle_vote_resp(self, frm: int, rejected: bool) -> int:
        return lib.qref_handle_vote_resp(ctypes.byref(self.c), frm, int(rejected))

    def candidate_resp(self, frm: int, rejected: bool, observer: bool, q: int) -> int:
        return lib.qref_candidate_vote_resp(ctypes.byref(self.c), frm, int(rejected),
                                            int(observer), q)


# ------------------------------------------------------------------------ batched forms -----
def commit_args(G, n_max, form, ring_len, match, committed_in, committed_out, last_index,
                term_start=None, term=None, ring=None, n_voting=None, changed=None,
                fallback=None, match_stride=None, term_mask=None) -> QrefCommitArgs:
    a = QrefCommitArgs()
    a.term_mask = None if term_mask is None else term_mask.ctypes.data
    a.G, a.n_max, a.form, a.ring_len = G, n_max, form, ring_len
    a.match_stride = G if match_stride is None else match_stride
    a.match = match.ctypes.data
    a.n_voting = None if n_voting is None else n_voting.ctypes.data
    a.committed_in = committed_in.ctypes.data
    a.committed_out = committed_out.ctypes.data
    a.last_index = last_index.ctypes.data
    a.term_start = None if term_start is None else term_start.ctypes.data
    a.term = None if term is None else term.ctypes.data
    a.ring = None if ring is None else ring.ctypes.data
    a.changed = None if changed is None else changed.ctypes.data
    a.fallback = None if fallback is None else fallback.ctypes.data
    return a


def commit_batch(a: QrefCommitArgs, nthreads: int = 1) -> int:
    return lib.qref_commit_batch(ctypes.byref(a), nthreads)


def words64(G):
    return (G + 63) // 64


def words32(G):
    return (G + 31) // 32


def readindex_batch(ack, n_voting, n_uniform, nthreads=1):
    G = len(ack)
    conf = np.zeros(words64(G), np.uint64)
    fb = np.zeros(words64(G), np.uint64)
    rc = lib.qref_readindex_batch(G, _ptr(ack), _ptr(n_voting), n_uniform, _ptr(conf), _ptr(fb),
                                  nthreads)
    assert rc == 0, rc
    return conf, fb


def vote_batch(granted, rejected, n_voting, n_uniform, nthreads=1):
    G = len(granted)
    out = np.zeros(words32(G), np.uint64)
    fb = np.zeros(words64(G), np.uint64)
    rc = lib.qref_vote_batch(G, _ptr(granted), _ptr(rejected), _ptr(n_voting), n_uniform,
                             _ptr(out), _ptr(fb), nthreads)
    assert rc == 0, rc
    return out, fb


def check_quorum_batch(active, n_voting, n_uniform, self_slot, nthreads=1):
    G = len(active)
    active = active.copy()
    hq = np.zeros(words64(G), np.uint64)
    fb = np.zeros(words64(G), np.uint64)
    rc = lib.qref_check_quorum_batch(G, _ptr(active), _ptr(n_voting), n_uniform, self_slot,
                                     _ptr(hq), _ptr(fb), nthreads)
    assert rc == 0, rc
    return hq, fb, active


# ------------------------------------------------------------------------ generator ---------
def spec(seed, G, n_max, cid_base=1, cid_stride=1, mixed_n=False, ring_len=16,
         parity_extras=False) -> QgenSpec:
    return QgenSpec(seed, G, cid_base, cid_stride, n_max, int(mixed_n), ring_len,
                    int(parity_extras))


class CommitInputs:
    """Host SoA commit inputs generated by qgen_commit (both term forms)."""

    def __init__(self, s: QgenSpec):
        G, n = s.G, s.n_max
        self.spec = s
        self.G, self.n_max, self.R = G, n, s.ring_len
        self.match = np.zeros(G * n, np.uint64)
        self.n_voting = np.zeros(G, np.uint8)
        self.committed_in = np.zeros(G, np.uint64)
        self.last_index = np.zeros(G, np.uint64)
        self.term_start = np.zeros(G, np.uint64)
        self.term = np.zeros(G, np.uint64)
        self.ring = np.zeros(G * s.ring_len, np.uint64)
        self.term_mask = np.zeros(G, np.uint16) if s.ring_len <= 16 else None
        a = commit_args(G, n, 0, s.ring_len, self.match, self.committed_in, self.committed_in,
                        self.last_index, self.term_start, self.term, self.ring, self.n_voting,
                        term_mask=self.term_mask)
        rc = lib.qgen_commit(ctypes.byref(s), ctypes.byref(a))
        assert rc == 0, rc

    def run(self, form: int, per_group_n: bool, nthreads: int = 1):
        """Oracle decision: returns (committed_out, changed, fallback, rc)."""
        G = self.G
        out = np.zeros(G, np.uint64)
        chg = np.zeros(words64(G), np.uint64)
        fb = np.zeros(words64(G), np.uint64)
        a = commit_args(G, self.n_max, form, self.R, self.match, self.committed_in, out,
                        self.last_index, self.term_start, self.term, self.ring,
                        self.n_voting if per_group_n else None, chg, fb,
                        term_mask=self.term_mask)
        rc = commit_batch(a, nthreads)
        return out, chg, fb, rc


class BitmapInputs:
    def __init__(self, s: QgenSpec):
        G = s.G
        self.spec = s
        self.G = G
        self.ack = np.zeros(G, np.uint8)
        self.granted = np.zeros(G, np.uint8)
        self.rejected = np.zeros(G, np.uint8)
        self.n_voting = np.zeros(G, np.uint8)
        rc = lib.qgen_bitmaps(ctypes.byref(s), _ptr(self.ack), _ptr(self.granted),
                              _ptr(self.rejected), _ptr(self.n_voting))
        assert rc == 0, rc


def readindex_multi_batch(ack_ordinal, ctx_index, n_pending, n_voting, n_uniform, K_max, n_max,
                          nthreads=1):
    """General multi-ctx ReadIndex: returns (released_index [K_max*G], released_count [G],
    fallback bitmap, batch_end [G]). ack_ordinal: uint16 [K_max][n_max][G]; ctx_index: uint64
    [K_max][G]."""
    G = len(ctx_index) // K_max
    rel = np.zeros(K_max * G, np.uint64)
    cnt = np.zeros(G, np.uint8)
    bend = np.zeros(G, np.uint8)
    fb = np.zeros(words64(G), np.uint64)
    rc = lib.qref_readindex_multi_batch(G, K_max, n_max, _ptr(ack_ordinal), _ptr(ctx_index),
                                        _ptr(n_pending), _ptr(n_voting), n_uniform, _ptr(rel),
                                        _ptr(cnt), _ptr(bend), _ptr(fb), nthreads)
    assert rc == 0, rc
    return rel, cnt, fb, bend


def c1_stream(seed: int, T: int, committed0: int, last0: int):
    """BASELINE config C1 stream: (match [3*T] slot-major, last [T])."""
    match = np.zeros(3 * T, np.uint64)
    last = np.zeros(T, np.uint64)
    assert lib.qgen_c1_stream(seed, T, committed0, last0, _ptr(match), _ptr(last)) == 0
    return match, last


def c1_run(match, last, term_start: int, committed0: int) -> np.ndarray:
    """Sequential raft.tryCommit over the C1 stream: committed after every step."""
    T = len(last)
    out = np.zeros(T, np.uint64)
    assert lib.qref_c1_run(T, _ptr(match), _ptr(last), term_start, committed0, _ptr(out)) == 0
    return out


def ingest_match(updates: np.ndarray, match: np.ndarray, stride: int, G: int, n_max: int) -> int:
    """updates: uint64 [count, 2] rows (group << 8 | slot, index); match updated in place."""
    u = np.ascontiguousarray(updates, np.uint64)
    return int(lib.qref_ingest_match(u.ctypes.data_as(_vp), len(u), match.ctypes.data_as(_vp),
                                     stride, G, n_max))


def ingest_ack(group_slot: np.ndarray, ack: np.ndarray, G: int, n_max: int) -> int:
    gs = np.ascontiguousarray(group_slot, np.uint64)
    return int(lib.qref_ingest_ack(gs.ctypes.data_as(_vp), len(gs), ack.ctypes.data_as(_vp), G,
                                   n_max))


def append(updates: np.ndarray, last_index, match_slot0, term_mask, ring_len: int, G: int) -> int:
    u = np.ascontiguousarray(updates, np.uint64)
    return int(lib.qref_append(u.ctypes.data_as(_vp), len(u), last_index.ctypes.data_as(_vp),
                               match_slot0.ctypes.data_as(_vp),
                               None if term_mask is None else term_mask.ctypes.data_as(_vp),
                               ring_len, G))


def fnv1a64(a: np.ndarray) -> int:
    a = np.ascontiguousarray(a)
    return int(lib.qref_fnv1a64(a.ctypes.data_as(_vp), a.nbytes))


class StepGroup:
    """One group replayed event by event through the reference's handlers (oracle/qref_step.c).
    Events are tuples: ("read", low, high) | ("msg", type, from, term, log_index, hint,
    hint_high, reject) | ("check_quorum",) | ("campaign",) | ("propose", n)."""

    def __init__(self, cluster_id, node_id, term, state, committed, last, term_start, members,
                 log=None):
        """log: None (the two-run history {(0, term - 1), (term_start, term)}) or
        (first_minus_1, [(start, term), ...]) — the node's log terms by index as runs
        (qref_group_set_log)."""
        self.c = Group()
        m = (Member * len(members))(*[Member(int(a), int(b), int(c), int(d))
                                      for a, b, c, d in members])
        rc = lib.qref_group_init(ctypes.byref(self.c), cluster_id, node_id, term, state,
                                 committed, last, term_start, m, len(members))
        assert rc == 0, rc
        if log is not None:
            first_minus_1, runs = log
            st = np.array([r[0] for r in runs], np.uint64)
            tm = np.array([r[1] for r in runs], np.uint64)
            rc = lib.qref_group_set_log(ctypes.byref(self.c), first_minus_1, len(runs),
                                        st.ctypes.data, tm.ctypes.data)
            assert rc == 0, (rc, log)
        self._out = StepOut()

    def log_terms(self):
        """(first_minus_1, [(start, term), ...]) of the group's log history now."""
        c = self.c
        return int(c.first_minus_1), [(int(c.run_start[k]), int(c.run_term[k]))
                                      for k in range(c.n_runs)]

    def __del__(self):
        if lib is not None and getattr(self, "c", None) is not None:
            lib.qref_group_free(ctypes.byref(self.c))

    def step(self, events):
        ev = (Event * max(1, len(events)))()
        for i, e in enumerate(events):
            k = e[0]
            if k == "read":
                ev[i] = Event(EV_READ, 19, 0, 0, 0, e[1], e[2], 0, 0)
            elif k == "msg":
                ev[i] = Event(EV_MSG, e[1], e[2], e[3], e[4], e[5], e[6], e[7], 0)
            elif k == "check_quorum":
                ev[i] = Event(EV_CHECK_QUORUM, 0, 0, 0, 0, 0, 0, 0, 0)
            elif k == "campaign":
                ev[i] = Event(EV_CAMPAIGN, 0, 0, 0, 0, 0, 0, 0, 0)
            elif k == "propose":
                ev[i] = Event(EV_PROPOSE, 0, 0, 0, e[1], 0, 0, 0, 0)
            else:
                raise ValueError(k)
        o = self._out
        rc = lib.qref_group_step(ctypes.byref(self.c), ev, len(events), ctypes.byref(o))
        if rc != 0:
            return rc
        return {
            "committed": int(o.committed), "commit_changed": bool(o.commit_changed),
            "ready": [(int(r.index), int(r.low), int(r.high)) for r in o.ready[:o.n_ready]],
            "resps": [(int(r.to), int(r.index), int(r.hint), int(r.hint_high))
                      for r in o.resps[:o.n_resps]],
            "states": [(int(r.term), int(r.state), int(r.reason)) for r in o.states[:o.n_states]],
            "dropped": [(int(r.low), int(r.high), int(r.from_), int(r.reason))
                        for r in o.dropped[:o.n_dropped]],
            "deferred": [int(x) for x in o.deferred[:o.n_deferred]],
        }

    def state(self):
        """(term, state, committed, last, term_start, [(node_id, match, role, active)],
        [(index, from, (low, high), n_confirmed)] in queue order)."""
        c = self.c
        members = [(int(m.node_id), int(m.match), int(m.role), int(m.active))
                   for m in c.members[:c.n_members]]
        reads = []
        ri = c.ri.contents if c.ri else None
        for qi in range(ri.n_queue if ri else 0):
            q = ri.queue[qi]
            for p in ri.pending[:ri.n_pending]:
                if p.ctx.low == q.low and p.ctx.high == q.high:
                    reads.append((int(p.index), int(p.from_), (int(q.low), int(q.high)),
                                  int(p.n_confirmed)))
        return (int(c.term), int(c.state), int(c.committed), int(c.last), int(c.term_start),
                members, reads)


class StepTotals(ctypes.Structure):
    _fields_ = [(k, _u64) for k in ("commits", "ready", "resps", "states", "dropped", "deferred",
                                    "committed_sum", "ready_digest", "commit_digest",
                                    "ready_order_digest")]


class StepBatch:
    """Many groups replayed event by event (qref_step_batch): the CPU baseline of the step
    worker, on the same compressed-row input (group index list, offsets, events) as
    hq_worker_step. Group records / members use the worker's numpy dtypes."""

    def __init__(self, groups: np.ndarray, members: np.ndarray):
        self.G = len(groups)
        self.h = lib.qref_groups_new(self.G)
        assert self.h
        rc = lib.qref_groups_init(self.h, self.G, _ptr(groups), _ptr(members))
        assert rc == 0, rc

    def close(self):
        if self.h:
            lib.qref_groups_free(self.h, self.G)
            self.h = None

    def committed(self, i: int) -> int:
        return int(Group.from_address(self.h + i * ctypes.sizeof(Group)).committed)

    def step(self, list_, offsets, events, nthreads=1):
        t = StepTotals()
        rc = lib.qref_step_batch(self.h, self.G, len(list_), _ptr(list_), _ptr(offsets),
                                 _ptr(events), nthreads, ctypes.byref(t))
        assert rc == 0, rc
        return {k: int(getattr(t, k)) for k, _ in StepTotals._fields_}
