"""Python binding of libhipquorum.so (include/hipquorum.h) via ctypes.

This is the harness-side caller of the C-ABI — the same entry points the Go cgo package
``internal/hipquorum`` binds. It adds no computation of its own: every decision
is made by the HIP kernels in ``dragonboat_amd/csrc``. There is no CPU fallback; if the shared
library is missing, importing this module raises.
"""
from __future__ import annotations

import ctypes
import os
from dataclasses import dataclass
from typing import Optional

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
# HQ_LIB_PATH: an alternative build of the same library (tuning experiments, tools/)
LIB_PATH = os.environ.get("HQ_LIB_PATH") or os.path.join(_HERE, "lib", "libhipquorum.so")

HQ_OK = 0
HQ_E_INVAL = -1
HQ_E_DEVICE = -2
HQ_E_NOMEM = -3
HQ_E_STATE = -4

HQ_MAX_VOTERS = 8
HQ_FORM_TERM_START = 0
HQ_FORM_TERM_RING = 1
HQ_FORM_TERM_MASK = 2
HQ_FORM_TERM_RING32 = 3
HQ_LAYOUT_COLUMNS = 0
HQ_LAYOUT_TILES = 1
HQ_LAYOUT_TILES_LEADER = 2   # tiles without the leader row: slot 0 = last_index
HQ_LAG_LEADER_IMPLICIT = 1   # hq_commit_lag_args.flags: lag rows start at slot 1
HQ_TILE_GROUPS = 128
HQ_LAYOUT_IN_PLACE = 0x100   # | HQ_LAYOUT_TILES_LEADER: a device-resident table decided in place
HQ_INGEST_GROUPED = 1        # hq_table_*: the records of one key are adjacent in the batch
HQ_INGEST_UNIQUE = 2         # hq_table_*: every key at most once in the batch
HQ_INGEST_ATOMIC = 4         # hq_table_ingest_*: the per-record atomic kernel, forced
HQ_INGEST_BINNED = 8         # hq_table_ingest_*: the two-pass binned kernels, forced
HQ_WORKER_ON_DEVICE = 1      # hq_worker_open_ex: the step worker's state and events on the GPU
HQ_WORKER_COMMIT_COLUMN = 2  # with it: a step's commits as a column when most groups commit
HQ_WORKER_COMMIT_ADVANCE = 4  # with it: commits as 4-byte advances when > 1/4 of groups commit
HQ_WORKER_READY_COMPACT = 8  # with it: ReadyToReads as 24-byte records (position, delta, ctx)
HQ_WORKER_READY_SLOTS = 16   # with it (+ COMMIT_ADVANCE): single ReadyToReads in per-tile slots
HQ_WAIT_BLOCK, HQ_WAIT_SLEEP, HQ_WAIT_SPIN, HQ_WAIT_CLOCK = 0, 1, 2, 0x100   # hq_worker_set_wait
HQ_WAIT_ADAPT = 3
SLOT_TILE = 256              # groups per ReadyToRead slot tile
HQ_ABI_VERSION = 21
HQ_ENGINE_SIGNAL = 1         # hq_engine_config.flags: per-step completion flags

OUTCOME_FOLLOWER = 0
OUTCOME_CANDIDATE = 1
OUTCOME_LEADER = 2

_u64p = ctypes.POINTER(ctypes.c_uint64)
_u8p = ctypes.POINTER(ctypes.c_uint8)
_vp = ctypes.c_void_p


class CommitArgs(ctypes.Structure):
    """Mirror of ``hq_commit_args``."""

    _fields_ = [
        ("G", ctypes.c_uint64),
        ("n_max", ctypes.c_uint32),
        ("form", ctypes.c_uint32),
        ("ring_len", ctypes.c_uint32),
        ("layout", ctypes.c_uint32),
        ("match_stride", ctypes.c_uint64),
        ("match", _vp),
        ("n_voting", _vp),
        ("committed_in", _vp),
        ("committed_out", _vp),
        ("last_index", _vp),
        ("term_start", _vp),
        ("term", _vp),
        ("ring", _vp),
        ("changed", _vp),
        ("fallback", _vp),
        ("term_mask", _vp),
        ("ring32", _vp),
    ]


class LagArgs(ctypes.Structure):
    """Mirror of ``hq_commit_lag_args``."""

    _fields_ = [
        ("G", ctypes.c_uint64),
        ("n_max", ctypes.c_uint32),
        ("form", ctypes.c_uint32),
        ("ring_len", ctypes.c_uint32),
        ("flags", ctypes.c_uint32),
        ("lag_stride", ctypes.c_uint64),
        ("lag", _vp),
        ("n_voting", _vp),
        ("cin_lag", _vp),
        ("cout_lag", _vp),
        ("ts_lag", _vp),
        ("lag_mask", _vp),
        ("changed", _vp),
        ("fallback", _vp),
    ]


class EngineConfig(ctypes.Structure):
    """Mirror of ``hq_engine_config``."""

    _fields_ = [(k, ctypes.c_uint32) for k in ("n_max", "form", "layout", "ring_len", "depth",
                                                "flags", "idle_us", "max_workgroups")]


class EngineStats(ctypes.Structure):
    """Mirror of ``hq_engine_stats``."""

    _fields_ = [("posted", ctypes.c_uint64), ("completed", ctypes.c_uint64),
                ("relaunches", ctypes.c_uint64), ("grid", ctypes.c_uint32),
                ("block", ctypes.c_uint32), ("depth", ctypes.c_uint32),
                ("running", ctypes.c_uint32)]


class SynthSpec(ctypes.Structure):
    """Mirror of ``hq_synth_spec``."""

    _fields_ = [
        ("seed", ctypes.c_uint64),
        ("G", ctypes.c_uint64),
        ("cid_base", ctypes.c_uint64),
        ("cid_stride", ctypes.c_uint64),
        ("n_max", ctypes.c_uint32),
        ("mixed_n", ctypes.c_uint32),
        ("ring_len", ctypes.c_uint32),
        ("parity_extras", ctypes.c_uint32),
    ]


# numpy mirrors of the packer structs (hq_member, hq_group_view, hq_msg)
ROLE_REMOTE, ROLE_OBSERVER, ROLE_WITNESS = 0, 1, 2
MEMBER_DTYPE = np.dtype([("node_id", "<u8"), ("match", "<u8"), ("role", "<u4"),
                         ("active", "<u4")], align=True)
GROUP_DTYPE = np.dtype([("node_id", "<u8"), ("committed", "<u8"), ("last_index", "<u8"),
                        ("term_start", "<u8"), ("term", "<u8"), ("ctx_low", "<u8"),
                        ("ctx_high", "<u8"), ("term_mask", "<u2"), ("reserved0", "<u2"),
                        ("reserved1", "<u4"), ("first_member", "<u4"), ("n_members", "<u4"),
                        ("first_msg", "<u4"), ("n_msgs", "<u4")], align=True)
MSG_DTYPE = np.dtype([("from", "<u8"), ("hint_low", "<u8"), ("hint_high", "<u8"),
                      ("reject", "<u4"), ("reserved", "<u4")], align=True)

# step worker records (include/hipquorum.h "step worker")
STATE_FOLLOWER, STATE_CANDIDATE, STATE_LEADER = 0, 1, 2
MSG_REPLICATE_RESP, MSG_REQUEST_VOTE_RESP, MSG_HEARTBEAT_RESP, MSG_READ_INDEX = 13, 15, 18, 19
EV_READ, EV_MESSAGE, EV_CHECK_QUORUM, EV_ELECTION, EV_PROPOSE = 1, 2, 3, 4, 5
REASON_VOTE, REASON_CHECK_QUORUM, REASON_HIGHER_TERM, REASON_CAMPAIGN = 1, 2, 3, 4
DROP_WITNESS, DROP_NOT_READY = 1, 2
EVENT_DTYPE = np.dtype([("kind", "<u4"), ("type", "<u4"), ("from", "<u8"), ("term", "<u8"),
                        ("log_index", "<u8"), ("hint", "<u8"), ("hint_high", "<u8"),
                        ("reject", "<u4"), ("reserved", "<u4")], align=True)
# hq_event16: a compact message record (hq_events16_encode_sized)
EVENT16_DTYPE = np.dtype([("kind", "u1"), ("type", "u1"), ("from", "<u2"), ("term", "<u4"),
                          ("value", "<u8")])
EV16_READ_CTX, EV16_FULL = 0x10, 0x80
WORKER_GROUP_DTYPE = np.dtype([("cluster_id", "<u8"), ("node_id", "<u8"), ("term", "<u8"),
                               ("committed", "<u8"), ("last_index", "<u8"), ("term_start", "<u8"),
                               ("state", "<u4"), ("n_members", "<u4"),
                               ("n_pending_reads", "<u4"), ("suspended", "<u4")], align=True)
READ_STATUS_DTYPE = np.dtype([("index", "<u8"), ("from", "<u8"), ("ctx_low", "<u8"),
                              ("ctx_high", "<u8"), ("n_confirmed", "<u4"), ("reserved", "<u4")],
                             align=True)
COMMIT_EVENT_DTYPE = np.dtype([("cluster_id", "<u8"), ("committed", "<u8")], align=True)
READY_DTYPE = np.dtype([("cluster_id", "<u8"), ("index", "<u8"), ("ctx_low", "<u8"),
                        ("ctx_high", "<u8")], align=True)
READY_COMPACT_DTYPE = np.dtype([("ctx_low", "<u8"), ("ctx_high", "<u8"), ("pos", "<u4"),
                                ("delta", "<i4")], align=True)
assert READY_COMPACT_DTYPE.itemsize == 24
READ_RESP_DTYPE = np.dtype([("cluster_id", "<u8"), ("to", "<u8"), ("log_index", "<u8"),
                            ("hint", "<u8"), ("hint_high", "<u8")], align=True)
STATE_CHANGE_DTYPE = np.dtype([("cluster_id", "<u8"), ("term", "<u8"), ("state", "<u4"),
                               ("reason", "<u4")], align=True)
DROPPED_READ_DTYPE = np.dtype([("cluster_id", "<u8"), ("ctx_low", "<u8"), ("ctx_high", "<u8"),
                               ("from", "<u8"), ("reason", "<u4"), ("reserved", "<u4")],
                              align=True)


# wire decode (include/hipquorum.h "wire decode")
HQ_RPC_BIN_VERSION = 210
WIRE_MESSAGE_DTYPE = np.dtype([("ev", EVENT_DTYPE), ("cluster_id", "<u8"), ("to", "<u8"),
                               ("log_term", "<u8"), ("commit", "<u8"), ("n_entries", "<u4"),
                               ("has_snapshot", "<u4")], align=True)


class WireBatchInfo(ctypes.Structure):
    _fields_ = [("n_messages", ctypes.c_uint64), ("deployment_id", ctypes.c_uint64),
                ("source_address_len", ctypes.c_uint64), ("bin_ver", ctypes.c_uint32),
                ("reserved", ctypes.c_uint32)]


class WireStats(ctypes.Structure):
    _fields_ = [(k, ctypes.c_uint64) for k in
                ("batches", "bytes", "messages", "entries", "snapshot_received",
                 "dropped_batches", "dropped_messages", "dropped_no_cluster")]


class StepInput(ctypes.Structure):
    """Mirror of ``hq_step_input``."""

    _fields_ = [("n_groups", ctypes.c_uint64), ("groups", _vp), ("offsets", _vp),
                ("events", _vp)]


class StepStream(ctypes.Structure):
    """Mirror of ``hq_step_stream``."""

    _fields_ = [("n_groups", ctypes.c_uint64), ("groups", _vp), ("offsets", _vp),
                ("boffsets", _vp), ("bytes", _vp), ("sizes", _vp), ("n_events", ctypes.c_uint64),
                ("n_bytes", ctypes.c_uint64), ("sizes16", _vp)]


class SizedStream(tuple):
    """A step's event stream in the sized form of ``hq_step_stream``: (groups, sizes, n_events,
    bytes), sizes[i] = events | bytes << 16 of group i (encode_events_sized) as uint32, or its
    byte count alone as uint16 (the 2-byte words, ``sizes16``)."""

    def __new__(cls, groups, sizes, n_events, data):
        return super().__new__(cls, (groups, sizes, n_events, data))


HQ_EVENT_STREAM_MAX = 64


class StepJob(ctypes.Structure):
    """Mirror of ``hq_step_job``."""

    _fields_ = [("worker", _vp), ("rows", _vp), ("stream", _vp), ("out", _vp),
                ("rc", ctypes.c_int), ("reserved", ctypes.c_int)]

STEP_OUTPUT_LISTS = [("commits", COMMIT_EVENT_DTYPE), ("ready", READY_DTYPE),
                     ("read_resps", READ_RESP_DTYPE), ("state_changes", STATE_CHANGE_DTYPE),
                     ("dropped_reads", DROPPED_READ_DTYPE), ("deferred", np.dtype("<u8")),
                     ("fallback_groups", np.dtype("<u8"))]


def expand_ready(compact, cluster_ids, committed_before):
    """HQ_WORKER_READY_COMPACT records -> READY_DTYPE records: cluster_ids[pos] and
    committed_before[pos] + delta (the listed groups' cluster ids and committed indexes before
    the step, in list order)."""
    out = np.zeros(len(compact), READY_DTYPE)
    pos = compact["pos"].astype(np.int64)
    out["cluster_id"] = np.asarray(cluster_ids, np.uint64)[pos]
    # (mod 2^64, as the device computed index - committed)
    out["index"] = np.asarray(committed_before, np.uint64)[pos] + \
        compact["delta"].astype(np.int64).astype(np.uint64)
    out["ctx_low"] = compact["ctx_low"]
    out["ctx_high"] = compact["ctx_high"]
    return out


class StepOutput(ctypes.Structure):
    """Mirror of ``hq_step_output``."""

    _fields_ = [f for name, _ in STEP_OUTPUT_LISTS
                for f in ((name, _vp), ("n_" + name, ctypes.c_uint64))] + \
               [("gpu_passes", ctypes.c_uint64), ("decisions", ctypes.c_uint64),
                ("handle_ns", ctypes.c_uint64), ("pass_ns", ctypes.c_uint64),
                ("pack_ns", ctypes.c_uint64), ("device_ns", ctypes.c_uint64),
                ("apply_ns", ctypes.c_uint64), ("committed_column", _vp),
                ("committed_advance", _vp), ("ready_compact", _vp),
                ("gpu_ns", ctypes.c_uint64), ("gpu_jobs", ctypes.c_uint32),
                ("wait_sleeps", ctypes.c_uint32), ("wait_poll_ns", ctypes.c_uint64),
                ("wait_sleep_ns", ctypes.c_uint64), ("wait_end_ns", ctypes.c_uint64),
                ("device_end_ticks", ctypes.c_uint64), ("ready_slots", _vp),
                ("ready_slot_counts", _vp), ("n_ready_tiles", ctypes.c_uint64),
                ("n_ready_slotted", ctypes.c_uint64), ("device_start_ticks", ctypes.c_uint64)]


# name -> (restype, argtypes); the complete export list of include/hipquorum.h
SIGNATURES = {
    "hq_abi_version": (ctypes.c_int, []),
    "hq_device_count": (ctypes.c_int, [ctypes.POINTER(ctypes.c_int)]),
    "hq_device_pci_bus_id": (ctypes.c_int, [ctypes.c_int, ctypes.c_char_p, ctypes.c_int]),
    "hq_pointer_kind": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(ctypes.c_int)]),
    "hq_open": (ctypes.c_int, [ctypes.c_int, ctypes.c_uint32, ctypes.POINTER(_vp)]),
    "hq_close": (None, [_vp]),
    "hq_last_error": (ctypes.c_char_p, [_vp]),
    "hq_sync": (ctypes.c_int, [_vp]),
    "hq_wait_for": (ctypes.c_int, [_vp, _vp]),
    "hq_malloc_dev": (ctypes.c_int, [_vp, ctypes.c_size_t, ctypes.POINTER(_vp)]),
    "hq_free_dev": (ctypes.c_int, [_vp, _vp]),
    "hq_alloc_pinned": (ctypes.c_int, [_vp, ctypes.c_size_t, ctypes.POINTER(_vp)]),
    "hq_free_pinned": (ctypes.c_int, [_vp, _vp]),
    "hq_memcpy_async": (ctypes.c_int, [_vp, _vp, _vp, ctypes.c_size_t, ctypes.c_int]),
    "hq_memset_async": (ctypes.c_int, [_vp, _vp, ctypes.c_int, ctypes.c_size_t]),
    "hq_timing_enable": (ctypes.c_int, [_vp, ctypes.c_int]),
    "hq_timing_begin_after": (ctypes.c_int, [_vp, ctypes.c_uint64]),
    "hq_timing_read": (ctypes.c_int, [_vp, ctypes.POINTER(ctypes.c_double), _u64p]),
    "hq_timing_reset": (ctypes.c_int, [_vp]),
    "hq_commit_dev": (ctypes.c_int, [_vp, ctypes.POINTER(CommitArgs)]),
    "hq_commit": (ctypes.c_int, [_vp, ctypes.POINTER(CommitArgs)]),
    "hq_commit_many_dev": (ctypes.c_int, [_vp, ctypes.POINTER(CommitArgs), ctypes.c_uint32]),
    "hq_commit_fused_dev": (ctypes.c_int, [_vp, ctypes.POINTER(CommitArgs), ctypes.c_uint32]),
    "hq_commit_lag_dev": (ctypes.c_int, [_vp, ctypes.POINTER(LagArgs)]),
    "hq_engine_open": (ctypes.c_int, [_vp, ctypes.POINTER(EngineConfig), ctypes.POINTER(_vp)]),
    "hq_engine_post": (ctypes.c_int, [_vp, ctypes.POINTER(CommitArgs), ctypes.c_uint32, _u64p]),
    "hq_engine_wait": (ctypes.c_int, [_vp, ctypes.c_uint64]),
    "hq_engine_drain": (ctypes.c_int, [_vp]),
    "hq_engine_run": (ctypes.c_int, [_vp, ctypes.POINTER(CommitArgs), ctypes.c_uint32, _u64p]),
    "hq_engine_timing": (ctypes.c_int, [_vp, _u64p, ctypes.POINTER(ctypes.c_double), ctypes.c_int]),
    "hq_engine_done_clock": (ctypes.c_int, [_vp, ctypes.c_uint64, _u64p]),
    "hq_engine_info": (ctypes.c_int, [_vp, ctypes.POINTER(EngineStats)]),
    "hq_engine_last_error": (ctypes.c_char_p, [_vp]),
    "hq_engine_dump": (ctypes.c_int, [_vp, ctypes.c_void_p, ctypes.c_uint32]),
    "hq_engine_close": (None, [_vp]),
    "hq_commit_lag_fused_dev": (ctypes.c_int, [_vp, ctypes.POINTER(LagArgs), ctypes.c_uint32]),
    "hq_pack_lags": (ctypes.c_int, [ctypes.c_uint64, ctypes.c_uint32, _vp, ctypes.c_uint64, _vp,
                                    _vp, _vp, _vp, ctypes.POINTER(LagArgs)]),
    "hq_unpack_lags": (ctypes.c_int, [ctypes.c_uint64, _vp, _vp, _vp, _vp]),
    "hq_readindex_dev": (ctypes.c_int, [_vp, ctypes.c_uint64, _vp, _vp, ctypes.c_uint32, _vp, _vp]),
    "hq_readindex": (ctypes.c_int, [_vp, ctypes.c_uint64, _vp, _vp, ctypes.c_uint32, _vp, _vp]),
    "hq_vote_dev": (ctypes.c_int, [_vp, ctypes.c_uint64, _vp, _vp, _vp, ctypes.c_uint32, _vp, _vp]),
    "hq_vote": (ctypes.c_int, [_vp, ctypes.c_uint64, _vp, _vp, _vp, ctypes.c_uint32, _vp, _vp]),
    "hq_readindex_vote_dev": (
        ctypes.c_int,
        [_vp, ctypes.c_uint64, _vp, _vp, _vp, _vp, ctypes.c_uint32, _vp, _vp, _vp],
    ),
    "hq_readindex_vote_tiles_dev": (
        ctypes.c_int,
        [_vp, ctypes.c_uint64, _vp, ctypes.c_uint32, ctypes.c_uint32, _vp, _vp, _vp],
    ),
    "hq_tile_bits_dev": (ctypes.c_int, [_vp, ctypes.c_uint64, _vp, _vp, _vp, _vp, _vp]),
    "hq_readindex_vote_tiles3_dev": (ctypes.c_int, [_vp, ctypes.c_uint64, _vp, _vp, _vp]),
    "hq_tile_bits3_dev": (ctypes.c_int, [_vp, ctypes.c_uint64, _vp, _vp, _vp, _vp,
                                         ctypes.c_uint32, _vp, _vp]),
    "hq_readindex_vote_planes_dev": (ctypes.c_int, [_vp, ctypes.c_uint64, _vp, _vp, _vp]),
    "hq_readindex_vote_cq_planes_dev": (ctypes.c_int, [_vp, ctypes.c_uint64, _vp, _vp, _vp,
                                                       _vp, _vp]),
    "hq_tile_planes_dev": (ctypes.c_int, [_vp, ctypes.c_uint64, _vp, _vp, _vp, _vp,
                                          ctypes.c_uint32, _vp, _vp]),
    "hq_tile_planes_host": (ctypes.c_int, [ctypes.c_uint64, _vp, _vp, _vp, _vp, ctypes.c_uint32,
                                           _vp, _vp]),
    "hq_tile_bits3_host": (ctypes.c_int, [ctypes.c_uint64, _vp, _vp, _vp, _vp, ctypes.c_uint32,
                                          _vp, _vp]),
    "hq_tile_bits_host": (ctypes.c_int, [ctypes.c_uint64, _vp, _vp, _vp, _vp, _vp]),
    "hq_check_quorum_planes_dev": (ctypes.c_int, [_vp, ctypes.c_uint64, _vp, ctypes.c_uint32,
                                                  _vp]),
    "hq_tile_cq_planes_dev": (ctypes.c_int, [_vp, ctypes.c_uint64, _vp, _vp, ctypes.c_uint32,
                                             ctypes.c_uint32, _vp, _vp]),
    "hq_tile_cq_planes_host": (ctypes.c_int, [ctypes.c_uint64, _vp, _vp, ctypes.c_uint32,
                                              ctypes.c_uint32, _vp, _vp]),
    "hq_check_quorum_dev": (
        ctypes.c_int,
        [_vp, ctypes.c_uint64, _vp, _vp, ctypes.c_uint32, ctypes.c_uint32, _vp, _vp],
    ),
    "hq_readindex_multi_dev": (ctypes.c_int, [_vp, ctypes.c_uint64, ctypes.c_uint32,
                                              ctypes.c_uint32, _vp, _vp, _vp, _vp,
                                              ctypes.c_uint32, _vp, _vp, _vp, _vp]),
    "hq_readindex_multi_tiles_dev": (ctypes.c_int, [_vp, ctypes.c_uint64, ctypes.c_uint32,
                                                    ctypes.c_uint32, _vp, ctypes.c_uint32,
                                                    ctypes.c_uint32, _vp, _vp, _vp, _vp]),
    "hq_tile_ri_multi_dev": (ctypes.c_int, [_vp, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint32,
                                            _vp, _vp, _vp, _vp, _vp]),
    "hq_ri_released_host": (ctypes.c_int, [ctypes.c_uint64, ctypes.c_uint32, _vp, _vp, _vp, _vp]),
    "hq_tile_ri_multi_host": (ctypes.c_int, [ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint32,
                                             _vp, _vp, _vp, _vp, _vp]),
    "hq_ingest_match_dev": (ctypes.c_int, [_vp, _vp, ctypes.c_uint64, _vp, ctypes.c_uint64,
                                           ctypes.c_uint64, ctypes.c_uint32, _vp]),
    "hq_ingest_ack_dev": (ctypes.c_int, [_vp, _vp, ctypes.c_uint64, _vp, ctypes.c_uint64,
                                         ctypes.c_uint32, _vp]),
    "hq_append_dev": (ctypes.c_int, [_vp, _vp, ctypes.c_uint64, _vp, _vp, _vp, ctypes.c_uint32,
                                     ctypes.c_uint64, _vp]),
    "hq_ingest_lag_dev": (ctypes.c_int, [_vp, _vp, ctypes.c_uint64, _vp, ctypes.c_uint64, _vp,
                                         ctypes.c_uint64, ctypes.c_uint32, _vp]),
    "hq_append_count_dev": (ctypes.c_int, [_vp, _vp, ctypes.c_uint64, _vp, _vp, _vp,
                                           ctypes.c_uint32, ctypes.c_uint64, _vp]),
    "hq_table_ingest_match_dev": (ctypes.c_int, [_vp, _vp, ctypes.c_uint64, _vp, ctypes.c_uint64,
                                                 ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32,
                                                 _vp]),
    "hq_table_ingest_lag_dev": (ctypes.c_int, [_vp, _vp, ctypes.c_uint64, _vp, ctypes.c_uint64,
                                               ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32,
                                               _vp]),
    "hq_table_append_dev": (ctypes.c_int, [_vp, _vp, ctypes.c_uint64, _vp, ctypes.c_uint64,
                                           ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32,
                                           ctypes.c_uint32, _vp]),
    "hq_table_append_count_dev": (ctypes.c_int, [_vp, _vp, ctypes.c_uint64, _vp, ctypes.c_uint64,
                                                 ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32,
                                                 ctypes.c_uint32, _vp]),
    "hq_table_committed_dev": (ctypes.c_int, [_vp, _vp, ctypes.c_uint64, ctypes.c_uint32,
                                              ctypes.c_uint32, _vp]),
    "hq_pack_commit": (ctypes.c_int, [_vp, ctypes.c_uint64, _vp, ctypes.POINTER(CommitArgs)]),
    "hq_pack_ring32": (ctypes.c_int, [_vp, ctypes.c_uint64, _vp]),
    "hq_tile_commit_dev": (ctypes.c_int, [_vp, ctypes.POINTER(CommitArgs), _vp]),
    "hq_tile_commit_host": (ctypes.c_int, [ctypes.POINTER(CommitArgs), _vp]),
    "hq_tile_commit_as_dev": (ctypes.c_int, [_vp, ctypes.POINTER(CommitArgs), _vp, ctypes.c_uint32]),
    "hq_tile_commit_as_host": (ctypes.c_int, [ctypes.POINTER(CommitArgs), _vp, ctypes.c_uint32]),
    "hq_pack_votes": (ctypes.c_int, [_vp, ctypes.c_uint64, _vp, _vp, _vp, _vp, _vp, _vp]),
    "hq_pack_acks": (ctypes.c_int, [_vp, ctypes.c_uint64, _vp, _vp, _vp, _vp, _vp,
                                    ctypes.c_uint32, _vp]),
    "hq_worker_open": (ctypes.c_int, [ctypes.c_int, ctypes.c_uint32, ctypes.POINTER(_vp)]),
    "hq_worker_open_ex": (ctypes.c_int, [ctypes.c_int, ctypes.c_uint32, ctypes.c_uint32,
                                         ctypes.POINTER(_vp)]),
    "hq_worker_close": (None, [_vp]),
    "hq_worker_last_error": (ctypes.c_char_p, [_vp]),
    "hq_worker_add_group": (ctypes.c_int, [_vp, _vp, _vp, ctypes.POINTER(ctypes.c_uint32)]),
    "hq_worker_set_group": (ctypes.c_int, [_vp, _vp, _vp]),
    "hq_worker_add_groups": (ctypes.c_int, [_vp, _vp, ctypes.c_uint64, _vp]),
    "hq_worker_find": (ctypes.c_int, [_vp, ctypes.c_uint64, ctypes.POINTER(ctypes.c_uint32)]),
    "hq_worker_get_group": (ctypes.c_int, [_vp, ctypes.c_uint64, _vp, _vp, ctypes.c_uint32, _vp,
                                           ctypes.c_uint32]),
    "hq_worker_step": (ctypes.c_int, [_vp, ctypes.POINTER(StepInput),
                                      ctypes.POINTER(StepOutput)]),
    "hq_worker_step_stream": (ctypes.c_int, [_vp, ctypes.POINTER(StepStream),
                                             ctypes.POINTER(StepOutput)]),
    "hq_worker_step_jobs": (ctypes.c_int, [_vp, ctypes.c_uint32]),
    "hq_events_encode": (ctypes.c_int, [ctypes.c_uint64, _vp, _vp, _vp, ctypes.c_uint64, _vp]),
    "hq_events_encode_sized": (ctypes.c_int, [ctypes.c_uint64, _vp, _vp, _vp, ctypes.c_uint64,
                                              _vp, _vp]),
    "hq_events16_encode_sized": (ctypes.c_int, [ctypes.c_uint64, _vp, _vp, _vp, ctypes.c_uint64,
                                                _vp, _vp, _vp, ctypes.c_uint32]),
    "hq_encode_stats_read": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int]),
    "hq_events16_encode_sized_multi": (ctypes.c_int, [_vp, ctypes.c_uint32, ctypes.c_uint32]),
    "hq_events_to16": (ctypes.c_int, [ctypes.c_uint64, _vp, _vp, _vp, ctypes.c_uint64, _vp]),
    "hq_events_decode": (ctypes.c_int, [ctypes.c_uint64, _vp, _vp, _vp, _vp]),
    "hq_events_count": (ctypes.c_int, [ctypes.c_uint64, _vp, _vp, _vp]),
    "hq_worker_set_wait": (ctypes.c_int, [_vp, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32]),
    "hq_wire_step_stream": (ctypes.c_int, [_vp, _vp, ctypes.POINTER(StepStream),
                                           ctypes.POINTER(WireStats)]),
    "hq_wire_decode_batch": (ctypes.c_int, [_vp, ctypes.c_size_t, _vp, ctypes.c_uint64, _u64p,
                                            ctypes.POINTER(WireBatchInfo)]),
    "hq_wire_open": (ctypes.c_int, [ctypes.c_uint64, ctypes.POINTER(_vp)]),
    "hq_wire_close": (None, [_vp]),
    "hq_wire_last_error": (ctypes.c_char_p, [_vp]),
    "hq_wire_reset": (ctypes.c_int, [_vp]),
    "hq_wire_add_local": (ctypes.c_int, [_vp, ctypes.c_uint64, _vp, ctypes.c_uint64]),
    "hq_wire_add_batch": (ctypes.c_int, [_vp, _vp, ctypes.c_size_t]),
    "hq_wire_step_input": (ctypes.c_int, [_vp, _vp, ctypes.POINTER(StepInput),
                                          ctypes.POINTER(WireStats)]),
    "hq_wire_attach": (ctypes.c_int, [_vp, _vp]),
    "hq_wire_encode_batch": (ctypes.c_int, [_vp, ctypes.c_uint64, ctypes.c_uint64, _vp,
                                            ctypes.c_size_t, _vp, ctypes.c_uint64, _u64p]),
    "hq_wire_add_locals": (ctypes.c_int, [_vp, ctypes.c_uint64, _vp, _vp, _vp]),
    "hq_wire_step_sized": (ctypes.c_int, [_vp, _vp, ctypes.c_uint64, _vp, ctypes.c_uint64,
                                          ctypes.POINTER(StepStream), ctypes.POINTER(WireStats)]),
    "hq_worker_group_count": (ctypes.c_int, [_vp, _u64p]),
    "hq_synth_commit_dev": (ctypes.c_int, [_vp, ctypes.POINTER(SynthSpec), ctypes.POINTER(CommitArgs)]),
    "hq_synth_commit_lag_dev": (ctypes.c_int, [_vp, ctypes.POINTER(SynthSpec),
                                               ctypes.POINTER(LagArgs), _vp]),
    "hq_synth_bitmaps_dev": (ctypes.c_int, [_vp, ctypes.POINTER(SynthSpec), _vp, _vp, _vp, _vp]),
}


def load_library(path: str = LIB_PATH) -> ctypes.CDLL:
    """Load libhipquorum.so and declare every exported signature. Raises if it is missing."""
    if not os.path.exists(path):
        raise ImportError(
            f"libhipquorum.so not found at {path}: build it with `make` (or "
            "__graft_entry__.build()); there is no CPU fallback for the quorum kernels"
        )
    lib = ctypes.CDLL(path)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    return lib


lib = load_library()


class HQError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"hipquorum error {code}: {msg}")
        self.code = code


def device_count() -> int:
    n = ctypes.c_int(0)
    lib.hq_device_count(ctypes.byref(n))
    return n.value


HQ_PTR_UNREGISTERED, HQ_PTR_PINNED_HOST, HQ_PTR_DEVICE = 0, 1, 2


def pointer_kind(a) -> int:
    """hq_pointer_kind of a numpy array's data (or a raw address / DeviceArray)."""
    p = a.ctypes.data if isinstance(a, np.ndarray) else getattr(a, "ptr", a)
    k = ctypes.c_int(0)
    _chk(lib.hq_pointer_kind(p, ctypes.byref(k)), "hq_pointer_kind")
    return k.value


def device_pci_bus_id(device: int) -> str:
    """hq_device_pci_bus_id: the PCI bus id of visible GPU `device` ("" if it has none)."""
    buf = ctypes.create_string_buffer(64)
    if lib.hq_device_pci_bus_id(device, buf, len(buf)) != HQ_OK:
        return ""
    return buf.value.decode()


@dataclass
class DeviceArray:
    """A device allocation owned by a Context (freed with it or by ``free``)."""

    ptr: int
    nbytes: int
    dtype: np.dtype
    count: int

    def at(self, elem_offset: int) -> int:
        return self.ptr + elem_offset * self.dtype.itemsize


class Context:
    """One hq_ctx: one HIP stream on one GPU (a step worker's handle, execengine.go:675-690)."""

    def __init__(self, device: int = 0):
        h = _vp()
        rc = lib.hq_open(device, 0, ctypes.byref(h))
        if rc != HQ_OK:
            raise HQError(rc, lib.hq_last_error(None).decode())
        self.h = h
        self.device = device
        self._allocs: dict[int, DeviceArray] = {}
        self._pinned: list[int] = []

    # -- lifetime ---------------------------------------------------------------------------
    def close(self) -> None:
        if self.h:
            lib.hq_sync(self.h)
            for a in list(self._allocs.values()):
                lib.hq_free_dev(self.h, _vp(a.ptr))
            self._allocs.clear()
            for p in self._pinned:
                lib.hq_free_pinned(self.h, _vp(p))
            self._pinned.clear()
            lib.hq_close(self.h)
            self.h = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def _check(self, rc: int) -> None:
        if rc != HQ_OK:
            raise HQError(rc, lib.hq_last_error(self.h).decode())

    # -- memory -----------------------------------------------------------------------------
    def empty(self, count: int, dtype) -> DeviceArray:
        dtype = np.dtype(dtype)
        p = _vp()
        self._check(lib.hq_malloc_dev(self.h, max(1, count * dtype.itemsize), ctypes.byref(p)))
        a = DeviceArray(p.value, count * dtype.itemsize, dtype, count)
        self._allocs[a.ptr] = a
        return a

    def free(self, a: Optional[DeviceArray]) -> None:
        if a is not None and a.ptr in self._allocs:
            del self._allocs[a.ptr]
            self._check(lib.hq_free_dev(self.h, _vp(a.ptr)))

    def upload(self, host: np.ndarray) -> DeviceArray:
        host = np.ascontiguousarray(host)
        a = self.empty(host.size, host.dtype)
        self._check(lib.hq_memcpy_async(self.h, _vp(a.ptr), host.ctypes.data_as(_vp), host.nbytes, 0))
        self.sync()
        return a

    def download(self, a: DeviceArray, count: Optional[int] = None) -> np.ndarray:
        count = a.count if count is None else count
        out = np.empty(count, dtype=a.dtype)
        self._check(lib.hq_memcpy_async(self.h, out.ctypes.data_as(_vp), _vp(a.ptr), out.nbytes, 1))
        self.sync()
        return out

    def pinned(self, count: int, dtype) -> np.ndarray:
        """A numpy view of pinned host memory (hq_alloc_pinned), freed with the context."""
        dtype = np.dtype(dtype)
        p = _vp()
        self._check(lib.hq_alloc_pinned(self.h, max(1, count * dtype.itemsize), ctypes.byref(p)))
        self._pinned.append(p.value)
        buf = (ctypes.c_char * (count * dtype.itemsize)).from_address(p.value)
        return np.frombuffer(buf, dtype=dtype, count=count)

    def h2d_async(self, dst: DeviceArray, src: np.ndarray) -> None:
        self._check(lib.hq_memcpy_async(self.h, _vp(dst.ptr), src.ctypes.data_as(_vp), src.nbytes, 0))

    def copy_to_ptr(self, dst_ptr: int, src: DeviceArray, nbytes: int) -> None:
        """Device-to-device copy into memory this context does not own (e.g. a torch tensor
        that a collective reads), asynchronous on the context's stream."""
        self._check(lib.hq_memcpy_async(self.h, _vp(dst_ptr), _vp(src.ptr), nbytes, 2))

    def d2h_async(self, dst: np.ndarray, src: DeviceArray) -> None:
        self._check(lib.hq_memcpy_async(self.h, dst.ctypes.data_as(_vp), _vp(src.ptr), dst.nbytes, 1))

    def memset(self, a: DeviceArray, value: int = 0) -> None:
        self._check(lib.hq_memset_async(self.h, _vp(a.ptr), value, a.nbytes))

    def sync(self) -> None:
        self._check(lib.hq_sync(self.h))

    def wait_for(self, other: "Context") -> None:
        """Order this context's stream after the work queued on ``other``'s (hq_wait_for)."""
        self._check(lib.hq_wait_for(self.h, other.h))

    # -- timing -----------------------------------------------------------------------------
    def timing(self, enable: bool) -> None:
        self._check(lib.hq_timing_enable(self.h, int(enable)))

    def timing_begin_after(self, launches: int) -> None:
        """Open a timed region behind the next ``launches`` launches (hq_timing_begin_after)."""
        self._check(lib.hq_timing_begin_after(self.h, launches))

    def timing_read(self) -> tuple[float, int]:
        ms = ctypes.c_double(0)
        n = ctypes.c_uint64(0)
        self._check(lib.hq_timing_read(self.h, ctypes.byref(ms), ctypes.byref(n)))
        return ms.value, n.value

    def timing_reset(self) -> None:
        self._check(lib.hq_timing_reset(self.h))

    # -- decisions (device pointers, asynchronous) -------------------------------------------
    def commit_dev(self, args: CommitArgs) -> None:
        self._check(lib.hq_commit_dev(self.h, ctypes.byref(args)))

    def commit_many_dev(self, batch) -> None:
        """batch: a ctypes array of CommitArgs (see ``commit_batch_array``)."""
        self._check(lib.hq_commit_many_dev(self.h, batch, len(batch)))

    def commit_fused_dev(self, batch) -> None:
        """The batches of ``batch`` (ctypes array of CommitArgs) in one launch when they can
        share it (hq_commit_fused_dev)."""
        self._check(lib.hq_commit_fused_dev(self.h, batch, len(batch)))

    def commit_lag_dev(self, args: LagArgs) -> None:
        self._check(lib.hq_commit_lag_dev(self.h, ctypes.byref(args)))

    def commit_lag_fused_dev(self, batch) -> None:
        """batch: a ctypes array of LagArgs (``lag_batch_array``)."""
        self._check(lib.hq_commit_lag_fused_dev(self.h, batch, len(batch)))

    def commit_host(self, args: CommitArgs) -> None:
        self._check(lib.hq_commit(self.h, ctypes.byref(args)))

    def tile_commit_dev(self, columns: CommitArgs, tiles, layout: int = HQ_LAYOUT_TILES) -> None:
        """hq_tile_commit_dev / hq_tile_commit_as_dev: the column batch's inputs cut into
        HQ_LAYOUT_TILES (or HQ_LAYOUT_TILES_LEADER) tiles."""
        if layout == HQ_LAYOUT_TILES:
            self._check(lib.hq_tile_commit_dev(self.h, ctypes.byref(columns), _p(tiles)))
        else:
            self._check(lib.hq_tile_commit_as_dev(self.h, ctypes.byref(columns), _p(tiles),
                                                  layout))

    def readindex_dev(self, G, ack, n_voting, n_uniform, confirmed, fallback=None) -> None:
        self._check(lib.hq_readindex_dev(self.h, G, _p(ack), _p(n_voting), n_uniform,
                                         _p(confirmed), _p(fallback)))

    def vote_dev(self, G, granted, rejected, n_voting, n_uniform, outcome, fallback=None) -> None:
        self._check(lib.hq_vote_dev(self.h, G, _p(granted), _p(rejected), _p(n_voting), n_uniform,
                                    _p(outcome), _p(fallback)))

    def readindex_vote_dev(self, G, ack, granted, rejected, n_voting, n_uniform, confirmed,
                           outcome, fallback=None) -> None:
        self._check(lib.hq_readindex_vote_dev(self.h, G, _p(ack), _p(granted), _p(rejected),
                                              _p(n_voting), n_uniform, _p(confirmed), _p(outcome),
                                              _p(fallback)))

    def readindex_vote_tiles_dev(self, G, tiles, per_group_n, n_uniform, confirmed, outcome,
                                 fallback=None) -> None:
        """hq_readindex_vote_tiles_dev: the fused pass over HQ_BITS_TILE_GROUPS-group tiles."""
        self._check(lib.hq_readindex_vote_tiles_dev(self.h, G, _p(tiles), int(per_group_n),
                                                    n_uniform, _p(confirmed), _p(outcome),
                                                    _p(fallback)))

    def tile_bits_dev(self, G, ack, granted, rejected, n_voting, tiles) -> None:
        """hq_tile_bits_dev: bitmap columns cut into tiles (rows [n] ack granted rejected)."""
        self._check(lib.hq_tile_bits_dev(self.h, G, _p(ack), _p(granted), _p(rejected),
                                         _p(n_voting), _p(tiles)))

    def readindex_vote_tiles3_dev(self, G, tiles, confirmed, outcome) -> None:
        self._check(lib.hq_readindex_vote_tiles3_dev(self.h, G, _p(tiles), _p(confirmed),
                                                     _p(outcome)))

    def tile_bits3_dev(self, G, ack, granted, rejected, n_voting, n_uniform, tiles,
                       fallback=None) -> None:
        self._check(lib.hq_tile_bits3_dev(self.h, G, _p(ack), _p(granted), _p(rejected),
                                          _p(n_voting), n_uniform, _p(tiles), _p(fallback)))

    def readindex_vote_planes_dev(self, G, planes, confirmed, outcome) -> None:
        self._check(lib.hq_readindex_vote_planes_dev(self.h, G, _p(planes), _p(confirmed),
                                                     _p(outcome)))

    def readindex_vote_cq_planes_dev(self, G, planes, active_planes, confirmed, outcome,
                                     has_quorum) -> None:
        """ReadIndex + vote + CheckQuorum in one launch (hq_readindex_vote_cq_planes_dev):
        active_planes as tile_cq_planes_dev(..., n_uniform=8, self_slot=0) builds them, zeroed
        in place."""
        self._check(lib.hq_readindex_vote_cq_planes_dev(self.h, G, _p(planes), _p(active_planes),
                                                        _p(confirmed), _p(outcome),
                                                        _p(has_quorum)))

    def tile_planes_dev(self, G, ack, granted, rejected, n_voting, n_uniform, planes,
                        fallback=None) -> None:
        self._check(lib.hq_tile_planes_dev(self.h, G, _p(ack), _p(granted), _p(rejected),
                                           _p(n_voting), n_uniform, _p(planes), _p(fallback)))

    def check_quorum_dev(self, G, active, n_voting, n_uniform, self_slot, has_quorum,
                         fallback=None) -> None:
        self._check(lib.hq_check_quorum_dev(self.h, G, _p(active), _p(n_voting), n_uniform,
                                            self_slot, _p(has_quorum), _p(fallback)))

    def check_quorum_planes_dev(self, G, planes, n_uniform, has_quorum) -> None:
        self._check(lib.hq_check_quorum_planes_dev(self.h, G, _p(planes), n_uniform,
                                                   _p(has_quorum)))

    def tile_cq_planes_dev(self, G, active, n_voting, n_uniform, self_slot, planes,
                           fallback=None) -> None:
        self._check(lib.hq_tile_cq_planes_dev(self.h, G, _p(active), _p(n_voting), n_uniform,
                                              self_slot, _p(planes), _p(fallback)))

    def readindex_host(self, G, ack, n_voting, n_uniform, confirmed, fallback=None) -> None:
        self._check(lib.hq_readindex(self.h, G, _p(ack), _p(n_voting), n_uniform, _p(confirmed),
                                     _p(fallback)))

    def vote_host(self, G, granted, rejected, n_voting, n_uniform, outcome, fallback=None) -> None:
        self._check(lib.hq_vote(self.h, G, _p(granted), _p(rejected), _p(n_voting), n_uniform,
                                _p(outcome), _p(fallback)))

    def readindex_multi_dev(self, G, K_max, n_max, ack_ordinal, ctx_index, n_pending, n_voting,
                            n_uniform, released_index, released_count, fallback=None,
                            batch_end=None):
        self._check(lib.hq_readindex_multi_dev(self.h, G, K_max, n_max, _p(ack_ordinal),
                                               _p(ctx_index), _p(n_pending), _p(n_voting),
                                               n_uniform, _p(released_index),
                                               _p(released_count), _p(batch_end),
                                               _p(fallback)))

    def readindex_multi_tiles_dev(self, G, K_max, n_max, tiles, flags, n_uniform, released_index,
                                  released_count, fallback=None, batch_end=None):
        """hq_readindex_multi_tiles_dev over 128-group tiles (tile_ri_multi_*)."""
        self._check(lib.hq_readindex_multi_tiles_dev(self.h, G, K_max, n_max, _p(tiles), flags,
                                                     n_uniform, _p(released_index),
                                                     _p(released_count), _p(batch_end),
                                                     _p(fallback)))

    def tile_ri_multi_dev(self, G, K_max, n_max, ack_ordinal, ctx_index, n_pending, n_voting,
                          tiles) -> None:
        self._check(lib.hq_tile_ri_multi_dev(self.h, G, K_max, n_max, _p(ack_ordinal),
                                             _p(ctx_index), _p(n_pending), _p(n_voting),
                                             _p(tiles)))

    def ingest_match_dev(self, updates, count, match, match_stride, G, n_max, n_skipped=None):
        """updates: device array of hq_match_update (uint64 pairs: group << 8 | slot, index)."""
        self._check(lib.hq_ingest_match_dev(self.h, _p(updates), count, _p(match), match_stride,
                                            G, n_max, _p(n_skipped)))

    def ingest_ack_dev(self, group_slot, count, ack, G, n_max, n_skipped=None):
        self._check(lib.hq_ingest_ack_dev(self.h, _p(group_slot), count, _p(ack), G, n_max,
                                          _p(n_skipped)))

    def append_dev(self, updates, count, last_index, match_slot0, term_mask, ring_len, G,
                   n_skipped=None):
        """updates: device array of hq_append_update (uint64 pairs: group, new_last)."""
        self._check(lib.hq_append_dev(self.h, _p(updates), count, _p(last_index),
                                      _p(match_slot0), _p(term_mask), ring_len, G,
                                      _p(n_skipped)))

    def ingest_lag_dev(self, updates, count, match, match_stride, last_index, G, n_max,
                       n_skipped=None):
        """updates: device uint64 array of group << 32 | slot << 28 | lag."""
        self._check(lib.hq_ingest_lag_dev(self.h, _p(updates), count, _p(match), match_stride,
                                          _p(last_index), G, n_max, _p(n_skipped)))

    def append_count_dev(self, updates, count, last_index, match_slot0, term_mask, ring_len, G,
                         n_skipped=None):
        """updates: device uint64 array of group << 32 | n_entries."""
        self._check(lib.hq_append_count_dev(self.h, _p(updates), count, _p(last_index),
                                            _p(match_slot0), _p(term_mask), ring_len, G,
                                            _p(n_skipped)))

    # -- device-resident progress table (HQ_LAYOUT_TILES_LEADER, decided in place) ----------
    def table_ingest_match_dev(self, updates, count, tiles, G, n_max, form, flags=0,
                               n_skipped=None):
        self._check(lib.hq_table_ingest_match_dev(self.h, _p(updates), count, _p(tiles), G, n_max,
                                                  form, flags, _p(n_skipped)))

    def table_ingest_lag_dev(self, updates, count, tiles, G, n_max, form, flags=0,
                             n_skipped=None):
        self._check(lib.hq_table_ingest_lag_dev(self.h, _p(updates), count, _p(tiles), G, n_max,
                                                form, flags, _p(n_skipped)))

    def table_append_dev(self, updates, count, tiles, G, n_max, form, ring_len=16, flags=0,
                         n_skipped=None):
        self._check(lib.hq_table_append_dev(self.h, _p(updates), count, _p(tiles), G, n_max, form,
                                            ring_len, flags, _p(n_skipped)))

    def table_append_count_dev(self, updates, count, tiles, G, n_max, form, ring_len=16, flags=0,
                               n_skipped=None):
        self._check(lib.hq_table_append_count_dev(self.h, _p(updates), count, _p(tiles), G, n_max,
                                                  form, ring_len, flags, _p(n_skipped)))

    def table_committed_dev(self, tiles, G, n_max, form, committed):
        self._check(lib.hq_table_committed_dev(self.h, _p(tiles), G, n_max, form, _p(committed)))

    def synth_commit_dev(self, spec: SynthSpec, args: CommitArgs) -> None:
        self._check(lib.hq_synth_commit_dev(self.h, ctypes.byref(spec), ctypes.byref(args)))

    def synth_commit_lag_dev(self, spec: SynthSpec, args: LagArgs, last_index=None) -> None:
        self._check(lib.hq_synth_commit_lag_dev(self.h, ctypes.byref(spec), ctypes.byref(args),
                                                _p(last_index)))

    def synth_bitmaps_dev(self, spec: SynthSpec, ack=None, granted=None, rejected=None,
                          n_voting=None) -> None:
        self._check(lib.hq_synth_bitmaps_dev(self.h, ctypes.byref(spec), _p(ack), _p(granted),
                                             _p(rejected), _p(n_voting)))


def _p(x) -> Optional[_vp]:
    """Pointer argument from a DeviceArray, a numpy array (host) or None."""
    if x is None:
        return None
    if isinstance(x, DeviceArray):
        return _vp(x.ptr)
    if isinstance(x, np.ndarray):
        return x.ctypes.data_as(_vp)
    if isinstance(x, int):
        return _vp(x)
    raise TypeError(f"unsupported pointer argument {type(x)}")


def _chk(rc: int, what: str) -> None:
    if rc != HQ_OK:
        raise HQError(rc, what)


def pack_commit(groups: np.ndarray, members: np.ndarray, n_max: int, ring_len: int = 16):
    """hq_pack_commit into fresh host SoA arrays; returns (dict of columns, fallback bitmap)."""
    G = len(groups)
    cols = dict(match=np.zeros(n_max * G, np.uint64), n_voting=np.zeros(G, np.uint8),
                committed_in=np.zeros(G, np.uint64), last_index=np.zeros(G, np.uint64),
                term_start=np.zeros(G, np.uint64), term=np.zeros(G, np.uint64),
                term_mask=np.zeros(G, np.uint16))
    fb = np.zeros(words64(G), np.uint64)
    a = CommitArgs()
    a.G, a.n_max, a.ring_len, a.match_stride = G, n_max, ring_len, G
    for k, v in cols.items():
        setattr(a, k, v.ctypes.data)
    a.fallback = fb.ctypes.data
    _chk(lib.hq_pack_commit(_p(groups), G, _p(members), ctypes.byref(a)), "hq_pack_commit")
    return cols, fb


def pack_ring32(ring: np.ndarray) -> np.ndarray:
    """hq_pack_ring32: the u32 ring of HQ_FORM_TERM_RING32 from a u64 term ring."""
    ring = np.ascontiguousarray(ring, np.uint64)
    out = np.zeros(len(ring), np.uint32)
    _chk(lib.hq_pack_ring32(_p(ring), len(ring), _p(out)), "hq_pack_ring32")
    return out


def lag_args(G, n_max, form, ring_len, lag, cin_lag, cout_lag, ts_lag=None, lag_mask=None,
             n_voting=None, changed=None, fallback=None, lag_stride=None) -> LagArgs:
    """LagArgs over device arrays / numpy arrays / raw pointers (see ``_p``)."""
    a = LagArgs()
    a.G, a.n_max, a.form, a.ring_len = G, n_max, form, ring_len
    a.lag_stride = G if lag_stride is None else lag_stride
    for name, v in (("lag", lag), ("cin_lag", cin_lag), ("cout_lag", cout_lag),
                    ("ts_lag", ts_lag), ("lag_mask", lag_mask), ("n_voting", n_voting),
                    ("changed", changed), ("fallback", fallback)):
        ptr = _p(v)
        setattr(a, name, ptr.value if ptr is not None else None)
    return a


def pack_lags(G, n_max, form, ring_len, match, committed, last_index, term_start=None,
              term_mask=None, match_stride=None, flags=0):
    """hq_pack_lags into fresh host arrays: (lag [rows*G] int32, cin_lag, ts_lag or lag_mask);
    rows = n_max, or n_max - 1 with flags = HQ_LAG_LEADER_IMPLICIT."""
    lag = np.zeros((n_max - (1 if flags & HQ_LAG_LEADER_IMPLICIT else 0)) * G, np.int32)
    cin = np.zeros(G, np.int32)
    ts = np.zeros(G, np.int32) if form == HQ_FORM_TERM_START else None
    lm = np.zeros(G, np.uint16) if form == HQ_FORM_TERM_MASK else None
    # (n_max = 1 with the leader flag has no lag row; the packer still wants a non-NULL lag
    # pointer and writes nothing through it)
    out = lag_args(G, n_max, form, ring_len, lag if lag.size else cin, cin, cin, ts, lm)
    out.flags = flags
    _chk(lib.hq_pack_lags(G, n_max, _p(np.ascontiguousarray(match, np.uint64)),
                          G if match_stride is None else match_stride,
                          _p(np.ascontiguousarray(committed, np.uint64)),
                          _p(np.ascontiguousarray(last_index, np.uint64)),
                          _p(None if term_start is None else np.ascontiguousarray(term_start, np.uint64)),
                          _p(None if term_mask is None else np.ascontiguousarray(term_mask, np.uint16)),
                          ctypes.byref(out)), "hq_pack_lags")
    return lag, cin, (ts if form == HQ_FORM_TERM_START else lm)


def unpack_lags(last_index: np.ndarray, cout_lag: np.ndarray, committed: np.ndarray,
                fallback: Optional[np.ndarray] = None) -> np.ndarray:
    """hq_unpack_lags: committed' = lastIndex - cout_lag for the groups without a fallback bit
    (updates ``committed`` in place and returns it)."""
    _chk(lib.hq_unpack_lags(len(last_index), _p(np.ascontiguousarray(last_index, np.uint64)),
                            _p(np.ascontiguousarray(cout_lag, np.int32)), _p(fallback),
                            _p(committed)), "hq_unpack_lags")
    return committed


def pack_votes(groups: np.ndarray, members: np.ndarray, msgs: np.ndarray):
    G = len(groups)
    gr, rj, nv = (np.zeros(G, np.uint8) for _ in range(3))
    fb = np.zeros(words64(G), np.uint64)
    _chk(lib.hq_pack_votes(_p(groups), G, _p(members), _p(msgs), _p(gr), _p(rj), _p(nv), _p(fb)),
         "hq_pack_votes")
    return gr, rj, nv, fb


def pack_acks(groups: np.ndarray, members: np.ndarray, msgs: np.ndarray, n_max: int = 8):
    G = len(groups)
    ack, act, nv = (np.zeros(G, np.uint8) for _ in range(3))
    fb = np.zeros(words64(G), np.uint64)
    _chk(lib.hq_pack_acks(_p(groups), G, _p(members), _p(msgs), _p(ack), _p(act), _p(nv), n_max,
                          _p(fb)), "hq_pack_acks")
    return ack, act, nv, fb


def commit_batch_array(args_list) -> ctypes.Array:
    arr = (CommitArgs * len(args_list))()
    for i, a in enumerate(args_list):
        arr[i] = a
    return arr


class Engine:
    """hq_engine_*: the persistent commit engine. One resident launch decides every batch posted
    to it (hq_commit_dev's decision bit for bit) with no launch boundary between steps; step
    workers post the way execEngine wakes them (execengine.go:115-123, 860-882)."""

    def __init__(self, ctx: Context, n_max: int, form: int, layout: int = HQ_LAYOUT_TILES_LEADER,
                 ring_len: int = 16, depth: int = 0, signal: bool = False, idle_us: int = 0,
                 max_workgroups: int = 0):
        cfg = EngineConfig(n_max=n_max, form=form, layout=layout, ring_len=ring_len, depth=depth,
                           flags=HQ_ENGINE_SIGNAL if signal else 0, idle_us=idle_us,
                           max_workgroups=max_workgroups)
        h = _vp()
        ctx._check(lib.hq_engine_open(ctx.h, ctypes.byref(cfg), ctypes.byref(h)))
        self.h = h
        self.ctx = ctx

    def _check(self, rc: int) -> None:
        if rc != HQ_OK:
            raise HQError(rc, lib.hq_engine_last_error(self.h).decode())

    def post(self, batch) -> int:
        """Post a ctypes array of CommitArgs (``commit_batch_array``) or one CommitArgs; returns
        the sequence number of the first posted step."""
        if isinstance(batch, CommitArgs):
            batch = commit_batch_array([batch])
        seq = ctypes.c_uint64(0)
        self._check(lib.hq_engine_post(self.h, batch, len(batch), ctypes.byref(seq)))
        return seq.value

    def wait(self, seq: int) -> None:
        self._check(lib.hq_engine_wait(self.h, seq))

    def dump(self) -> dict:
        """hq_engine_dump: the device-side state (diagnostic)."""
        n = 8 + 16384
        buf = (ctypes.c_uint64 * n)()
        self._check(lib.hq_engine_dump(self.h, buf, n))
        head = ("posted", "relayed", "polled", "exit_epoch", "launches", "grid", "completed",
                "running")
        out = {k: int(buf[i]) for i, k in enumerate(head)}
        out["cursor"] = np.frombuffer(buf, np.uint64, out["grid"], 8 * 8).copy()
        depth = self.info().depth
        arr = np.frombuffer(buf, np.uint64, 9 * depth, 8 * (8 + out["grid"])).copy()
        out["arrive"] = arr[:8 * depth].reshape(depth, 8)
        out["top"] = arr[8 * depth:]
        return out

    def drain(self) -> None:
        self._check(lib.hq_engine_drain(self.h))

    def run(self, batch) -> int:
        """hq_engine_run: post the batches and drain, the STOP handed over with the steps when
        no grid is resident (one launch that ends at its last step); returns the first seq."""
        seq = ctypes.c_uint64(0)
        self._check(lib.hq_engine_run(self.h, batch, len(batch), ctypes.byref(seq)))
        return seq.value

    def timing(self, reset: bool = False) -> tuple[int, float]:
        """(finished resident launches, their total GPU ms) since the last reset."""
        n = ctypes.c_uint64(0)
        ms = ctypes.c_double(0)
        self._check(lib.hq_engine_timing(self.h, ctypes.byref(n), ctypes.byref(ms), int(reset)))
        return n.value, ms.value

    def done_clock(self, seq: int) -> int:
        t = ctypes.c_uint64(0)
        self._check(lib.hq_engine_done_clock(self.h, seq, ctypes.byref(t)))
        return t.value

    def info(self) -> EngineStats:
        st = EngineStats()
        self._check(lib.hq_engine_info(self.h, ctypes.byref(st)))
        return st

    def close(self) -> None:
        if self.h:
            lib.hq_engine_close(self.h)
            self.h = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()


def pack_lag_updates(group, slot, lag) -> np.ndarray:
    """8-byte match deltas for hq_ingest_lag_dev (lag < 2^28, slot < 16)."""
    g, s, l = (np.asarray(x, np.uint64) for x in (group, slot, lag))
    if (l >= np.uint64(1 << 28)).any() or (s >= np.uint64(16)).any():
        raise ValueError("lag >= 2^28 or slot >= 16: use the 16-byte hq_match_update form")
    return (g << np.uint64(32)) | (s << np.uint64(28)) | l


def pack_append_counts(group, n) -> np.ndarray:
    """8-byte appends for hq_append_count_dev (n entries, 1 <= n < 2^32)."""
    return (np.asarray(group, np.uint64) << np.uint64(32)) | np.asarray(n, np.uint64)


def lag_batch_array(args_list) -> ctypes.Array:
    arr = (LagArgs * len(args_list))()
    for i, a in enumerate(args_list):
        arr[i] = a
    return arr


def words64(G: int) -> int:
    return (G + 63) // 64


def commit_tile_words(n_max: int, form: int, layout: int = HQ_LAYOUT_TILES) -> int:
    """hq_commit_tile_words(_for): u64 words of one tile of HQ_TILE_GROUPS groups."""
    if layout == HQ_LAYOUT_TILES_LEADER:
        n_max -= 1
    if form == HQ_FORM_TERM_MASK:
        return (n_max + 2) * HQ_TILE_GROUPS + 32
    return (n_max + 3) * HQ_TILE_GROUPS


def commit_tiles(G: int) -> int:
    return (G + HQ_TILE_GROUPS - 1) // HQ_TILE_GROUPS


def tile_commit_host(columns: CommitArgs, layout: int = HQ_LAYOUT_TILES) -> np.ndarray:
    """hq_tile_commit_host / hq_tile_commit_as_host over host column arrays (pointers in
    ``columns``): the tiles as a uint64 array."""
    out = np.zeros(commit_tiles(columns.G) *
                   commit_tile_words(columns.n_max, columns.form, layout), np.uint64)
    if layout == HQ_LAYOUT_TILES:
        _chk(lib.hq_tile_commit_host(ctypes.byref(columns), _p(out)), "hq_tile_commit_host")
    else:
        _chk(lib.hq_tile_commit_as_host(ctypes.byref(columns), _p(out), layout),
             "hq_tile_commit_as_host")
    return out


class TileView:
    """Group-order access to the rows of HQ_LAYOUT_TILES(_LEADER) tiles held in a host uint64
    array (tests and host-side re-syncs; the kernels read the tiles directly). Row position 2i of
    tile t holds group 128 t + i, position 2i + 1 group 128 t + 64 + i (include/hipquorum.h)."""

    def __init__(self, tiles: np.ndarray, G: int, n_max: int, form: int, layout: int):
        lay = layout & 0xFF
        self.tiles, self.G, self.n_max, self.form = tiles, G, n_max, form
        self.lead = lay == HQ_LAYOUT_TILES_LEADER
        self.nr = n_max - 1 if self.lead else n_max      # match rows
        self.tw = commit_tile_words(n_max, form, lay)
        g = np.arange(G, dtype=np.int64)
        i = g % HQ_TILE_GROUPS
        self.base = (g // HQ_TILE_GROUPS) * self.tw
        self.pos = 2 * (i % 64) + i // 64
        self.rows = {"committed": self.nr, "last_index": self.nr + 1, "aux": self.nr + 2}

    def _idx(self, row: int, groups=None):
        b = self.base if groups is None else self.base[groups]
        p = self.pos if groups is None else self.pos[groups]
        return b + row * HQ_TILE_GROUPS + p

    def row(self, name: str) -> np.ndarray:
        """committed / last_index (u64) or aux (term_start / term u64, or the u16 term mask)."""
        r = self.rows[name]
        if name == "aux" and self.form == HQ_FORM_TERM_MASK:
            return self.tiles.view(np.uint16)[4 * (self.base + r * HQ_TILE_GROUPS) + self.pos]
        return self.tiles[self._idx(r)]

    def match(self) -> np.ndarray:
        """match slot-major [n_max][G]; with the leader layout slot 0 is lastIndex."""
        out = np.empty((self.n_max, self.G), np.uint64)
        s0 = 0
        if self.lead:
            out[0] = self.row("last_index")
            s0 = 1
        for s in range(s0, self.n_max):
            out[s] = self.tiles[self._idx(s - s0)]
        return out

    def set_row(self, name: str, groups, values) -> None:
        r = self.rows[name]
        if name == "aux" and self.form == HQ_FORM_TERM_MASK:
            self.tiles.view(np.uint16)[4 * (self.base[groups] + r * HQ_TILE_GROUPS)
                                       + self.pos[groups]] = values
        else:
            self.tiles[self._idx(r, groups)] = values


def tile_view(tiles: np.ndarray, G: int, n_max: int, form: int, layout: int) -> TileView:
    return TileView(tiles, G, n_max, form, layout)


HQ_BITS_TILE_GROUPS = 1024


def bits_tiles(G: int) -> int:
    return (G + HQ_BITS_TILE_GROUPS - 1) // HQ_BITS_TILE_GROUPS


def bits_tile_bytes(G: int, per_group_n: bool) -> int:
    """Bytes of the bitmap tiles of G groups (rows [n] ack granted rejected, 1024 bytes each)."""
    return bits_tiles(G) * (4 if per_group_n else 3) * HQ_BITS_TILE_GROUPS


def tile_bits_host(ack, granted, rejected, n_voting=None) -> np.ndarray:
    """hq_tile_bits_host over host uint8 columns: the tiles as a uint8 array."""
    G = len(ack)
    cols = [np.ascontiguousarray(a, np.uint8) if a is not None else None
            for a in (ack, granted, rejected, n_voting)]
    out = np.empty(bits_tile_bytes(G, n_voting is not None), np.uint8)
    _chk(lib.hq_tile_bits_host(G, *[_p(c) for c in cols], _p(out)), "hq_tile_bits_host")
    return out


def tile_bits3_host(ack, granted, rejected, n_voting=None, n_uniform=0):
    """hq_tile_bits3_host over host uint8 columns: (tiles uint8 array, fallback words)."""
    G = len(ack)
    cols = [np.ascontiguousarray(a, np.uint8) if a is not None else None
            for a in (ack, granted, rejected, n_voting)]
    out = np.empty(bits_tiles(G) * 3 * HQ_BITS_TILE_GROUPS, np.uint8)
    fb = np.zeros(words64(G), np.uint64)
    _chk(lib.hq_tile_bits3_host(G, *[_p(c) for c in cols], n_uniform, _p(out), _p(fb)),
         "hq_tile_bits3_host")
    return out, fb


HQ_PLANE_TILE_GROUPS = 2048
HQ_RI_TILE_GROUPS = 128
HQ_RI_TILE_PER_K = 1
HQ_RI_TILE_PER_N = 2


def ri_tile_bytes(K_max: int, n_max: int, flags: int) -> int:
    return K_max * n_max * 256 + K_max * 1024 + (128 if flags & HQ_RI_TILE_PER_K else 0) + \
        (128 if flags & HQ_RI_TILE_PER_N else 0)


def tile_ri_multi_host(G, K_max, n_max, ack_ordinal, ctx_index, n_pending=None, n_voting=None):
    """hq_tile_ri_multi_host: (tiles uint8 array, flags) of host columns."""
    flags = (HQ_RI_TILE_PER_K if n_pending is not None else 0) | \
        (HQ_RI_TILE_PER_N if n_voting is not None else 0)
    ntiles = (G + HQ_RI_TILE_GROUPS - 1) // HQ_RI_TILE_GROUPS
    out = np.zeros(ntiles * ri_tile_bytes(K_max, n_max, flags), np.uint8)
    cols = [np.ascontiguousarray(ack_ordinal, np.uint16), np.ascontiguousarray(ctx_index, np.uint64),
            None if n_pending is None else np.ascontiguousarray(n_pending, np.uint8),
            None if n_voting is None else np.ascontiguousarray(n_voting, np.uint8)]
    _chk(lib.hq_tile_ri_multi_host(G, K_max, n_max, *[_p(c) for c in cols], _p(out)),
         "hq_tile_ri_multi_host")
    return out, flags


def ri_released_host(K_max, ctx_index, released_count, batch_end):
    """hq_ri_released_host: released_index uint64 [K_max][G] from the compact outputs of
    readindex_multi(_tiles)_dev with released_index None, and the caller's ctx_index."""
    cnt = np.ascontiguousarray(released_count, np.uint8)
    G = len(cnt)
    idx = np.ascontiguousarray(ctx_index, np.uint64).reshape(-1)
    be = np.ascontiguousarray(batch_end, np.uint8)
    if len(idx) != K_max * G or len(be) != G:
        raise ValueError("ri_released_host: ctx_index [K_max][G], batch_end [G]")
    out = np.empty(K_max * G, np.uint64)
    _chk(lib.hq_ri_released_host(G, K_max, _p(idx), _p(cnt), _p(be), _p(out)),
         "hq_ri_released_host")
    return out


def plane_tiles(G: int) -> int:
    return (G + HQ_PLANE_TILE_GROUPS - 1) // HQ_PLANE_TILE_GROUPS


def cq_plane_bytes(G: int, n_uniform: int) -> int:
    """hq_cq_plane_bytes: CheckQuorum planes of G groups (n_uniform 0 = per-group n)."""
    return plane_tiles(G) * (n_uniform - 1 if n_uniform else 10) * (HQ_PLANE_TILE_GROUPS // 8)


def tile_cq_planes_host(active, n_voting=None, n_uniform=0, self_slot=0):
    """hq_tile_cq_planes_host over a host uint8 active column: (planes uint8, fallback words)."""
    G = len(active)
    act = np.ascontiguousarray(active, np.uint8)
    nv = None if n_voting is None else np.ascontiguousarray(n_voting, np.uint8)
    out = np.empty(max(1, cq_plane_bytes(G, 0 if nv is not None else n_uniform)), np.uint8)
    fb = np.zeros(words64(G), np.uint64)
    _chk(lib.hq_tile_cq_planes_host(G, _p(act), _p(nv), n_uniform, self_slot, _p(out), _p(fb)),
         "hq_tile_cq_planes_host")
    return out[:cq_plane_bytes(G, 0 if nv is not None else n_uniform)], fb


def tile_planes_host(ack, granted, rejected, n_voting=None, n_uniform=0):
    """hq_tile_planes_host over host uint8 columns: (planes uint8 array, fallback words)."""
    G = len(ack)
    cols = [np.ascontiguousarray(a, np.uint8) if a is not None else None
            for a in (ack, granted, rejected, n_voting)]
    out = np.empty(plane_tiles(G) * 3 * HQ_PLANE_TILE_GROUPS, np.uint8)
    fb = np.zeros(words64(G), np.uint64)
    _chk(lib.hq_tile_planes_host(G, *[_p(c) for c in cols], n_uniform, _p(out), _p(fb)),
         "hq_tile_planes_host")
    return out, fb


def words32(G: int) -> int:
    return (G + 31) // 32


# ------------------------------------------------------------------------------ device buffers
@dataclass
class CommitBuffers:
    """SoA device state of one batch of G groups (DESIGN.md "Data layout in HBM")."""

    G: int
    n_max: int
    form: int
    ring_len: int
    match: DeviceArray
    committed_in: DeviceArray
    committed_out: DeviceArray
    last_index: DeviceArray
    ring: Optional[DeviceArray]
    n_voting: Optional[DeviceArray]
    changed: DeviceArray
    fallback: DeviceArray
    term_start: Optional[DeviceArray] = None
    term: Optional[DeviceArray] = None
    term_mask: Optional[DeviceArray] = None
    ring32: Optional[DeviceArray] = None
    tiles: Optional[DeviceArray] = None    # HQ_LAYOUT_TILES(_LEADER) copy of the input columns
    tile_layout: int = HQ_LAYOUT_TILES

    def args(self) -> CommitArgs:
        a = CommitArgs()
        a.G = self.G
        a.n_max = self.n_max
        a.form = self.form
        a.ring_len = self.ring_len
        a.match_stride = self.G
        a.match = self.match.ptr
        a.n_voting = self.n_voting.ptr if self.n_voting else None
        a.committed_in = self.committed_in.ptr
        a.committed_out = self.committed_out.ptr
        a.last_index = self.last_index.ptr
        a.term_start = self.term_start.ptr if self.term_start else None
        a.term = self.term.ptr if self.term else None
        a.ring = self.ring.ptr if self.ring else None
        a.changed = self.changed.ptr
        a.fallback = self.fallback.ptr
        a.term_mask = self.term_mask.ptr if self.term_mask else None
        a.ring32 = self.ring32.ptr if self.ring32 else None
        return a

    def tile_args(self) -> CommitArgs:
        """The same batch in its tile layout: the inputs from ``tiles`` (filled by
        ``Context.tile_commit_dev(b.args(), b.tiles, b.tile_layout)``), outputs as in ``args``."""
        a = self.args()
        a.layout = self.tile_layout
        a.match = self.tiles.ptr
        a.match_stride = 0
        a.committed_in = a.last_index = a.term_start = a.term = a.term_mask = None
        return a

    def arrays(self):
        return [x for x in (self.match, self.committed_in, self.committed_out, self.last_index,
                            self.term_start, self.term, self.ring, self.term_mask, self.n_voting,
                            self.changed, self.fallback, self.ring32, self.tiles)
                if x is not None]


def alloc_commit(ctx: Context, G: int, n_max: int, form: int, ring_len: int = 16,
                 per_group_n: bool = False, with_both_aux: bool = False,
                 tiled: bool = False, tile_layout: int = HQ_LAYOUT_TILES) -> CommitBuffers:
    """Allocate the SoA columns of one commit batch (match is slot-major [n_max][G]).
    with_both_aux allocates the columns of all four term forms (to compare them); tiled adds
    the tile buffer of the form in ``tile_layout`` (HQ_LAYOUT_TILES or _TILES_LEADER)."""
    need_ts = form == HQ_FORM_TERM_START or with_both_aux
    need_ring = form == HQ_FORM_TERM_RING or with_both_aux
    need_ring32 = form == HQ_FORM_TERM_RING32 or with_both_aux
    need_mask = form == HQ_FORM_TERM_MASK or (with_both_aux and ring_len <= 16)
    b = CommitBuffers(
        G=G, n_max=n_max, form=form, ring_len=ring_len,
        match=ctx.empty(G * n_max, np.uint64),
        committed_in=ctx.empty(G, np.uint64),
        committed_out=ctx.empty(G, np.uint64),
        last_index=ctx.empty(G, np.uint64),
        ring=ctx.empty(G * ring_len, np.uint64) if need_ring else None,
        n_voting=ctx.empty(G, np.uint8) if per_group_n else None,
        changed=ctx.empty(words64(G), np.uint64),
        fallback=ctx.empty(words64(G), np.uint64),
        term_start=ctx.empty(G, np.uint64) if need_ts else None,
        term=ctx.empty(G, np.uint64) if need_ring or need_ring32 else None,
        term_mask=ctx.empty(G, np.uint16) if need_mask else None,
        ring32=ctx.empty(G * ring_len, np.uint32) if need_ring32 else None,
        tiles=ctx.empty(commit_tiles(G) * commit_tile_words(n_max, form, tile_layout), np.uint64)
        if tiled else None,
        tile_layout=tile_layout,
    )
    return b


@dataclass
class LagBuffers:
    """Device lag-layout state of one batch (hq_commit_lag_args)."""

    G: int
    n_max: int
    form: int
    ring_len: int
    lag: DeviceArray
    cin_lag: DeviceArray
    cout_lag: DeviceArray
    aux: DeviceArray          # ts_lag (int32) or lag_mask (uint16)
    changed: DeviceArray
    fallback: DeviceArray
    last_index: Optional[DeviceArray] = None
    stride: int = 0           # lag row stride (G rounded up to 4: 16-byte aligned rows)

    def args(self, leader_implicit: bool = False) -> LagArgs:
        """leader_implicit: the same batch with HQ_LAG_LEADER_IMPLICIT, the lag rows viewed
        from slot 1 (the generator writes every row; slot 0's lag is 0 by construction)."""
        ts = self.aux if self.form == HQ_FORM_TERM_START else None
        lm = self.aux if self.form == HQ_FORM_TERM_MASK else None
        stride = self.stride or self.G
        a = lag_args(self.G, self.n_max, self.form, self.ring_len, self.lag, self.cin_lag,
                     self.cout_lag, ts, lm, None, self.changed, self.fallback, lag_stride=stride)
        if leader_implicit:
            a.flags = HQ_LAG_LEADER_IMPLICIT
            a.lag = self.lag.ptr + stride * 4
        return a

    def arrays(self):
        return [x for x in (self.lag, self.cin_lag, self.cout_lag, self.aux, self.changed,
                            self.fallback, self.last_index) if x is not None]


def alloc_commit_lag(ctx: Context, G: int, n_max: int, form: int, ring_len: int = 16,
                     with_last: bool = False) -> LagBuffers:
    stride = (G + 3) & ~3
    return LagBuffers(
        G=G, n_max=n_max, form=form, ring_len=ring_len, stride=stride,
        lag=ctx.empty(stride * n_max, np.int32), cin_lag=ctx.empty(G, np.int32),
        cout_lag=ctx.empty(G, np.int32),
        aux=ctx.empty(G, np.int32 if form == HQ_FORM_TERM_START else np.uint16),
        changed=ctx.empty(words64(G), np.uint64), fallback=ctx.empty(words64(G), np.uint64),
        last_index=ctx.empty(G, np.uint64) if with_last else None)


def synth_spec(seed: int, G: int, n_max: int, cid_base: int = 1, cid_stride: int = 1,
               mixed_n: bool = False, ring_len: int = 16, parity_extras: bool = False) -> SynthSpec:
    s = SynthSpec()
    s.seed = seed
    s.G = G
    s.cid_base = cid_base
    s.cid_stride = cid_stride
    s.n_max = n_max
    s.mixed_n = int(mixed_n)
    s.ring_len = ring_len
    s.parity_extras = int(parity_extras)
    return s


def free_commit(ctx: Context, b: CommitBuffers) -> None:
    for a in b.arrays():
        ctx.free(a)


class Worker:
    """The step worker (hq_worker_*): one step's events in, the reference's step results out,
    every quorum decision taken by the kernels."""

    def __init__(self, device: int = 0, n_max: int = 8, on_device: bool = False,
                 commit_column: bool = False, commit_advance: bool = False,
                 ready_compact: bool = False, ready_slots: bool = False):
        """on_device: HQ_WORKER_ON_DEVICE, the group state resident on the GPU and every event
        taken there (hq_dstep.hip); otherwise the host worker (events on the host, decisions
        in GPU passes). commit_column: HQ_WORKER_COMMIT_COLUMN (results carry
        'committed_column' instead of 'commits' when most listed groups commit);
        commit_advance: HQ_WORKER_COMMIT_ADVANCE ('committed_advance', u32 per listed group,
        when more than a quarter of them commit); ready_compact: HQ_WORKER_READY_COMPACT (results
        carry 'ready_compact', READY_COMPACT_DTYPE, instead of 'ready'; expand_ready rebuilds
        the records); ready_slots: HQ_WORKER_READY_SLOTS (with commit_advance: a sized stream
        step's single ReadyToReads come as 'ready_slots', READY_COMPACT_DTYPE in group order,
        out of the list; merge_ready rebuilds the step's whole list)."""
        self.h = _vp()
        flags = (HQ_WORKER_ON_DEVICE if on_device else 0) | \
            (HQ_WORKER_COMMIT_COLUMN if commit_column else 0) | \
            (HQ_WORKER_COMMIT_ADVANCE if commit_advance else 0) | \
            (HQ_WORKER_READY_COMPACT if ready_compact else 0) | \
            (HQ_WORKER_READY_SLOTS if ready_slots else 0)
        rc = lib.hq_worker_open_ex(device, n_max, flags, ctypes.byref(self.h))
        if rc != HQ_OK:
            raise HQError(rc, "hq_worker_open: " + lib.hq_last_error(None).decode())
        self.n_max = n_max
        self.on_device = on_device

    def close(self) -> None:
        if self.h:
            lib.hq_worker_close(self.h)
            self.h = _vp()

    def set_wait(self, mode: int = HQ_WAIT_BLOCK, poll_us: int = 50, sleep_us: int = 20,
                 clock: bool = False) -> None:
        """hq_worker_set_wait: how the worker's thread waits for its device step."""
        self._check(lib.hq_worker_set_wait(self.h, mode | (HQ_WAIT_CLOCK if clock else 0),
                                           poll_us, sleep_us), "hq_worker_set_wait")

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def _check(self, rc: int, what: str) -> None:
        if rc != HQ_OK:
            raise HQError(rc, f"{what}: {lib.hq_worker_last_error(self.h).decode()}")

    @staticmethod
    def _group(cluster_id, node_id, term, state, committed, last_index, term_start, members):
        g = np.zeros(1, WORKER_GROUP_DTYPE)
        g["cluster_id"], g["node_id"], g["term"], g["state"] = cluster_id, node_id, term, state
        g["committed"], g["last_index"], g["term_start"] = committed, last_index, term_start
        m = np.asarray(members, MEMBER_DTYPE)
        g["n_members"] = len(m)
        return g, m

    def add_group(self, cluster_id, node_id, term, state, committed, last_index, term_start,
                  members) -> int:
        """Adds a group; returns its handle."""
        g, m = self._group(cluster_id, node_id, term, state, committed, last_index, term_start,
                           members)
        h = ctypes.c_uint32()
        self._check(lib.hq_worker_add_group(self.h, _p(g), _p(m), ctypes.byref(h)),
                    "hq_worker_add_group")
        return h.value

    def find(self, cluster_id) -> int:
        h = ctypes.c_uint32()
        self._check(lib.hq_worker_find(self.h, cluster_id, ctypes.byref(h)), "hq_worker_find")
        return h.value

    def set_group(self, cluster_id, node_id, term, state, committed, last_index, term_start,
                  members) -> None:
        g, m = self._group(cluster_id, node_id, term, state, committed, last_index, term_start,
                           members)
        self._check(lib.hq_worker_set_group(self.h, _p(g), _p(m)), "hq_worker_set_group")

    def get_group(self, cluster_id):
        """(group record, members, pending reads) of one group."""
        g = np.zeros(1, WORKER_GROUP_DTYPE)
        self._check(lib.hq_worker_get_group(self.h, cluster_id, _p(g), None, 0, None, 0),
                    "hq_worker_get_group")
        m = np.zeros(int(g["n_members"][0]), MEMBER_DTYPE)
        r = np.zeros(int(g["n_pending_reads"][0]), READ_STATUS_DTYPE)
        self._check(lib.hq_worker_get_group(self.h, cluster_id, _p(g), _p(m), len(m), _p(r),
                                            len(r)), "hq_worker_get_group")
        return g[0], m, r

    def step(self, groups, offsets, events, copy=True):
        """One step: `groups` (uint32 handles), `offsets` (uint64, len(groups) + 1) and
        `events` (EVENT_DTYPE). Returns a dict of numpy record arrays plus counters; with
        copy=False the arrays are views of the worker's buffers, valid until its next call."""
        groups = np.ascontiguousarray(groups, np.uint32)
        offsets = np.ascontiguousarray(offsets, np.uint64)
        events = np.ascontiguousarray(events, EVENT_DTYPE)
        assert len(offsets) == len(groups) + 1
        inp = StepInput(len(groups), _p(groups), _p(offsets), _p(events))
        out = StepOutput()
        self._check(lib.hq_worker_step(self.h, ctypes.byref(inp), ctypes.byref(out)),
                    "hq_worker_step")
        return self._results(out, copy, len(groups))

    def step_stream(self, groups, offsets, boffsets, data, copy=True):
        """hq_worker_step_stream: the step's events as an event stream (encode_events)."""
        groups = np.ascontiguousarray(groups, np.uint32)
        offsets = np.ascontiguousarray(offsets, np.uint64)
        boffsets = np.ascontiguousarray(boffsets, np.uint64)
        data = np.ascontiguousarray(data, np.uint8)
        assert len(offsets) == len(groups) + 1 == len(boffsets)
        inp = StepStream(len(groups), _p(groups), _p(offsets), _p(boffsets),
                         _p(data) if len(data) else None)
        out = StepOutput()
        self._check(lib.hq_worker_step_stream(self.h, ctypes.byref(inp), ctypes.byref(out)),
                    "hq_worker_step_stream")
        return self._results(out, copy, len(groups))

    def step_sized(self, groups, sizes, n_events, data, copy=True):
        """hq_worker_step_stream in the sized form (encode_events_sized): per-group size words
        instead of the two prefix arrays."""
        inp, keep = _sized_input(groups, sizes, n_events, data)
        out = StepOutput()
        self._check(lib.hq_worker_step_stream(self.h, ctypes.byref(inp), ctypes.byref(out)),
                    "hq_worker_step_stream")
        del keep
        return self._results(out, copy, len(sizes))

    @staticmethod
    def _results(out, copy, n_listed=0):
        res = {}
        for name, dt in STEP_OUTPUT_LISTS:
            n = getattr(out, "n_" + name)
            ptr = getattr(out, name)
            if n == 0 or (name == "commits" and (out.committed_column or out.committed_advance)) \
                    or (name == "ready" and out.ready_compact):
                res[name] = np.zeros(0, dt)
                continue
            buf = (ctypes.c_char * (n * dt.itemsize)).from_address(ptr)
            res[name] = np.frombuffer(buf, dt).copy() if copy else np.frombuffer(buf, dt)
        for k in ("gpu_passes", "decisions", "handle_ns", "pass_ns", "pack_ns", "device_ns",
                  "apply_ns", "gpu_ns", "gpu_jobs", "wait_sleeps", "wait_poll_ns",
                  "wait_sleep_ns", "wait_end_ns", "device_end_ticks", "device_start_ticks"):
            res[k] = getattr(out, k)
        if out.ready_slots:
            # tile t's records at slots[256 t ..], counts[t] of them: gathered in tile order (=
            # group order)
            nt = out.n_ready_tiles
            cnt = np.frombuffer((ctypes.c_char * (4 * nt)).from_address(out.ready_slot_counts),
                                np.uint32).astype(np.int64)
            allr = np.frombuffer((ctypes.c_char * (nt * SLOT_TILE * READY_COMPACT_DTYPE.itemsize))
                                 .from_address(out.ready_slots), READY_COMPACT_DTYPE)
            keep = np.arange(SLOT_TILE)[None, :] < cnt[:, None]
            res["ready_slots"] = allr.reshape(nt, SLOT_TILE)[keep]   # (a copy, tile order)
            assert len(res["ready_slots"]) == out.n_ready_slotted
        if out.committed_column:
            buf = (ctypes.c_char * (n_listed * 8)).from_address(out.committed_column)
            col = np.frombuffer(buf, np.uint64)
            res["committed_column"] = col.copy() if copy else col
            res["n_commits"] = out.n_commits
        if out.committed_advance:
            buf = (ctypes.c_char * (n_listed * 4)).from_address(out.committed_advance)
            col = np.frombuffer(buf, np.uint32)
            res["committed_advance"] = col.copy() if copy else col
            res["n_commits"] = out.n_commits
        if out.ready_compact:
            n = out.n_ready
            buf = (ctypes.c_char * (n * READY_COMPACT_DTYPE.itemsize)).from_address(out.ready_compact)
            rc = np.frombuffer(buf, READY_COMPACT_DTYPE)
            res["ready_compact"] = rc.copy() if copy else rc
        return res

    def add_groups(self, groups: np.ndarray, members: np.ndarray) -> None:
        """Bulk add: WORKER_GROUP_DTYPE records, members of consecutive groups back to back."""
        groups = np.ascontiguousarray(groups, WORKER_GROUP_DTYPE)
        members = np.ascontiguousarray(members, MEMBER_DTYPE)
        assert int(groups["n_members"].sum()) == len(members)
        self._check(lib.hq_worker_add_groups(self.h, _p(groups), len(groups), _p(members)),
                    "hq_worker_add_groups")


class StepJobs:
    """hq_worker_step_jobs over prepared jobs: jobs = [(worker, (groups, offsets, events))]
    (rows) or [(worker, (groups, offsets, boffsets, bytes))] (event stream). run() steps them
    at once on native threads and returns one result dict per job (as Worker.step)."""

    def __init__(self, jobs):
        self.jobs = jobs
        self.keep, self.arr = [], (StepJob * len(jobs))()
        self.outs = [StepOutput() for _ in jobs]
        for j, (w, a) in enumerate(jobs):
            if isinstance(a, SizedStream):
                inp, keep = _sized_input(*a)
                self.arr[j].stream = ctypes.cast(ctypes.pointer(inp), _vp)
                self.keep += keep + [inp]
            elif len(a) == 3:
                g, o, e = (np.ascontiguousarray(a[0], np.uint32),
                           np.ascontiguousarray(a[1], np.uint64),
                           np.ascontiguousarray(a[2], EVENT_DTYPE))
                inp = StepInput(len(g), _p(g), _p(o), _p(e))
                self.arr[j].rows = ctypes.cast(ctypes.pointer(inp), _vp)
                self.keep += [g, o, e, inp]
            else:
                g, o, b, d = (np.ascontiguousarray(a[0], np.uint32),
                              np.ascontiguousarray(a[1], np.uint64),
                              np.ascontiguousarray(a[2], np.uint64),
                              np.ascontiguousarray(a[3], np.uint8))
                inp = StepStream(len(g), _p(g), _p(o), _p(b), _p(d) if len(d) else None)
                self.arr[j].stream = ctypes.cast(ctypes.pointer(inp), _vp)
                self.keep += [g, o, b, d, inp]
            self.arr[j].worker = w.h
            self.arr[j].out = ctypes.cast(ctypes.pointer(self.outs[j]), _vp)

    def execute(self):
        """The native call alone (hq_worker_step_jobs); results() then reads the outputs."""
        rc = lib.hq_worker_step_jobs(self.arr, len(self.jobs))
        if rc != HQ_OK:
            bad = [j for j in range(len(self.jobs)) if self.arr[j].rc != HQ_OK]
            msg = lib.hq_worker_last_error(self.jobs[bad[0]][0].h).decode() if bad \
                else "a worker listed twice"
            raise HQError(rc, f"hq_worker_step_jobs: {msg}")

    def results(self, copy=True):
        """One result dict per job (as Worker.step) of the last execute()."""
        return [Worker._results(o, copy, len(a[1]) if isinstance(a, SizedStream) else len(a[0]))
                for o, (_, a) in zip(self.outs, self.jobs)]

    def run(self, copy=True):
        self.execute()
        return self.results(copy)


def step_jobs(jobs, copy=True):
    """StepJobs(jobs).run(copy)."""
    return StepJobs(jobs).run(copy)


def encode_events(offsets, events):
    """hq_events_encode: (stream bytes as uint8, boffsets) of rows grouped by `offsets`."""
    offsets = np.ascontiguousarray(offsets, np.uint64)
    events = np.ascontiguousarray(events, EVENT_DTYPE)
    n = len(offsets) - 1
    ne = int(offsets[-1] - offsets[0]) if n > 0 else 0
    out = np.zeros(max(1, ne * HQ_EVENT_STREAM_MAX), np.uint8)
    boff = np.zeros(n + 1, np.uint64)
    _chk(lib.hq_events_encode(n, _p(offsets), _p(events) if len(events) else None, _p(out),
                              len(out), _p(boff)), "hq_events_encode")
    return out[:int(boff[-1])].copy(), boff


def _sized_input(groups, sizes, n_events, data):
    """groups None: the step lists the worker's handles 0 .. len(sizes) - 1; uint16 sizes are the
    2-byte words (bytes only), any other dtype the 4-byte words."""
    s16 = getattr(sizes, "dtype", None) == np.uint16
    z = np.ascontiguousarray(sizes, np.uint16 if s16 else np.uint32)
    g = None if groups is None else np.ascontiguousarray(groups, np.uint32)
    d = np.ascontiguousarray(data, np.uint8)
    assert g is None or len(g) == len(z)
    inp = StepStream(len(z), _p(g), None, None, _p(d) if len(d) else None,
                     None if s16 else _p(z), int(n_events), len(d), _p(z) if s16 else None)
    return inp, [g, z, d]


def sizes16_of(sizes):
    """The 2-byte words (bytes only) of 4-byte size words."""
    return (np.asarray(sizes, np.uint32) >> np.uint32(16)).astype(np.uint16)


def count_events(boffsets, data):
    """hq_events_count: the event prefix (uint64, len(boffsets)) of a stream's groups."""
    boffsets = np.ascontiguousarray(boffsets, np.uint64)
    data = np.ascontiguousarray(data, np.uint8)
    n = len(boffsets) - 1
    off = np.zeros(n + 1, np.uint64)
    _chk(lib.hq_events_count(n, _p(boffsets), _p(data) if len(data) else None, _p(off)),
         "hq_events_count")
    return off


def merge_ready(res, cluster_ids, committed_before):
    """A step's ReadyToReads (READY_DTYPE) in the reference's order (group order), whatever form
    the worker returned them in: the list ('ready' or 'ready_compact') and, with
    HQ_WORKER_READY_SLOTS, the slots ('ready_slots'), merged by group position as the Go
    EachReady walks them: each slot record goes before the first list record of a later group,
    so both sequences keep their own order (a misordered list stays misordered). cluster_ids and
    committed_before: the listed groups' in list order; a 32-byte list record's position is found
    from its cluster id."""
    cids = np.asarray(cluster_ids, np.uint64)
    lst, lpos = np.zeros(0, READY_DTYPE), np.zeros(0, np.int64)
    if "ready_compact" in res:
        rc = res["ready_compact"]
        lst, lpos = expand_ready(rc, cids, committed_before), rc["pos"].astype(np.int64)
    elif len(res.get("ready", ())):
        lst = res["ready"]
        order = np.argsort(cids, kind="stable")
        lpos = order[np.searchsorted(cids, lst["cluster_id"], sorter=order)].astype(np.int64)
        assert np.array_equal(cids[lpos], lst["cluster_id"])
    if "ready_slots" not in res or len(res["ready_slots"]) == 0:
        return np.asarray(lst)
    rs = res["ready_slots"]
    slots = expand_ready(rs, cids, committed_before)
    if len(lst) == 0:
        return slots
    # (the first list record past a slot's group: past the running maximum of the list's
    # positions, which is non-decreasing)
    at = np.searchsorted(np.maximum.accumulate(lpos), rs["pos"].astype(np.int64), "right")
    return np.insert(np.asarray(lst), at, slots)


def encode_events_sized(offsets, events):
    """hq_events_encode_sized: (stream bytes as uint8, per-group size words) of rows grouped by
    `offsets`."""
    offsets = np.ascontiguousarray(offsets, np.uint64)
    events = np.ascontiguousarray(events, EVENT_DTYPE)
    n = len(offsets) - 1
    ne = int(offsets[-1] - offsets[0]) if n > 0 else 0
    out = np.zeros(max(1, ne * HQ_EVENT_STREAM_MAX), np.uint8)
    sizes = np.zeros(max(0, n), np.uint32)
    nb = ctypes.c_uint64(0)
    _chk(lib.hq_events_encode_sized(n, _p(offsets), _p(events) if len(events) else None,
                                    _p(out), len(out), _p(sizes), ctypes.byref(nb)),
         "hq_events_encode_sized")
    return out[:nb.value].copy(), sizes


def events_to16(offsets, events):
    """hq_events_to16: (compact records as EVENT16_DTYPE, their per-group offsets) of rows
    grouped by `offsets`."""
    offsets = np.ascontiguousarray(offsets, np.uint64)
    events = np.ascontiguousarray(events, EVENT_DTYPE)
    n = len(offsets) - 1
    ne = int(offsets[-1] - offsets[0]) if n > 0 else 0
    out = np.zeros(max(1, 5 * ne), EVENT16_DTYPE)
    off16 = np.zeros(n + 1, np.uint64)
    _chk(lib.hq_events_to16(n, _p(offsets), _p(events) if len(events) else None, _p(out),
                            len(out), _p(off16)), "hq_events_to16")
    return out[:int(off16[-1])].copy(), off16


def encode_events16_sized_into(offsets16, recs, out: np.ndarray, sizes: np.ndarray,
                               threads: int = 1):
    """hq_events16_encode_sized into caller buffers (`out` uint8, `sizes` uint32 of
    len(offsets16) - 1, both contiguous): returns (n_events, n_bytes); `threads` native threads."""
    n = len(offsets16) - 1
    assert offsets16.dtype == np.uint64 and recs.dtype == EVENT16_DTYPE
    assert out.dtype == np.uint8 and sizes.dtype == np.uint32 and len(sizes) >= n
    assert offsets16.flags.c_contiguous and recs.flags.c_contiguous and out.flags.c_contiguous
    ne, nb = ctypes.c_uint64(0), ctypes.c_uint64(0)
    _chk(lib.hq_events16_encode_sized(n, _p(offsets16), _p(recs) if len(recs) else None,
                                      _p(out), len(out), _p(sizes), ctypes.byref(ne),
                                      ctypes.byref(nb), threads), "hq_events16_encode_sized")
    return ne.value, nb.value


class Encode16Job(ctypes.Structure):
    """hq_encode16_job (include/hipquorum.h)."""
    _fields_ = [("n_groups", ctypes.c_uint64), ("offsets16", _vp), ("recs", _vp), ("out", _vp),
                ("cap", ctypes.c_uint64), ("sizes", _vp), ("n_events", ctypes.c_uint64),
                ("n_bytes", ctypes.c_uint64), ("rc", ctypes.c_int), ("reserved", ctypes.c_int),
                ("sizes16", _vp)]


class Encode16Batch:
    """A reusable hq_events16_encode_sized_multi call over fixed buffers: jobs =
    [(offsets16, recs, out, sizes)] as encode_events16_sized_into's arguments, whose contents may
    change between calls (a producer refilling the same receive buffers step after step) but
    not their places. The job table is built once, so a call is one C call: building it per call
    cost ~25 us of Python per job (400 us for 16 workers' streams)."""

    def __init__(self, jobs):
        self._jobs = list(jobs)              # (keeps the arrays alive)
        self.n = len(self._jobs)
        self.arr = (Encode16Job * max(1, self.n))()
        for b, (off, recs, out, sizes) in zip(self.arr, self._jobs):
            n = len(off) - 1
            assert off.dtype == np.uint64 and recs.dtype == EVENT16_DTYPE
            assert out.dtype == np.uint8 and sizes.dtype in (np.uint32, np.uint16)
            assert len(sizes) >= n
            assert off.flags.c_contiguous and recs.flags.c_contiguous and out.flags.c_contiguous
            b.n_groups, b.offsets16 = n, _p(off)
            b.recs = _p(recs) if len(recs) else None
            b.out, b.cap = _p(out), len(out)
            if sizes.dtype == np.uint16:     # the 2-byte words (hq_step_stream.sizes16)
                b.sizes16 = _p(sizes)
            else:
                b.sizes = _p(sizes)
        self._addr = ctypes.addressof(self.arr)

    def run(self, threads: int = 1):
        """Encode every job; returns [(n_events, n_bytes)] per job."""
        rc = lib.hq_events16_encode_sized_multi(self._addr, self.n, threads)
        if rc:
            for j, b in enumerate(self.arr[:self.n]):
                if b.rc:
                    raise HQError(b.rc, f"hq_events16_encode_sized_multi job {j}")
            _chk(rc, "hq_events16_encode_sized_multi")
        return [(b.n_events, b.n_bytes) for b in self.arr[:self.n]]


def encode_events16_sized_multi(jobs, threads: int = 1):
    """hq_events16_encode_sized_multi: jobs = [(offsets16, recs, out, sizes)] as
    encode_events16_sized_into's arguments, encoded in one call whose `threads` native threads
    split the records of all jobs evenly; returns [(n_events, n_bytes)] per job."""
    return Encode16Batch(jobs).run(threads)


ENCODE_STATS_FIELDS = ("calls", "tasks", "helped", "wall_ns", "encode_ns", "copy_ns", "lag_ns",
                       "max_lag_ns", "run_ns")


def encode_stats(reset: bool = False) -> dict:
    """hq_encode_stats_read: the threaded encodes' phase clocks (process-wide sums)."""
    buf = (ctypes.c_uint64 * len(ENCODE_STATS_FIELDS))()
    _chk(lib.hq_encode_stats_read(ctypes.addressof(buf), 1 if reset else 0),
         "hq_encode_stats_read")
    return dict(zip(ENCODE_STATS_FIELDS, (int(x) for x in buf)))


def encode_events16_sized(offsets16, recs, threads: int = 1):
    """hq_events16_encode_sized: (stream bytes as uint8, per-group size words, n_events)."""
    offsets16 = np.ascontiguousarray(offsets16, np.uint64)
    recs = np.ascontiguousarray(recs, EVENT16_DTYPE)
    n = len(offsets16) - 1
    out = np.zeros(max(1, len(recs) * HQ_EVENT_STREAM_MAX), np.uint8)
    sizes = np.zeros(max(0, n), np.uint32)
    ne, nb = encode_events16_sized_into(offsets16, recs, out, sizes, threads)
    return out[:nb].copy(), sizes, ne


def encode_events_sized_into(offsets, events, out: np.ndarray, sizes: np.ndarray) -> int:
    """hq_events_encode_sized into caller buffers (a producer writing the stream straight into
    its pinned receive buffer): `out` uint8, `sizes` uint32 of len(offsets) - 1, both contiguous.
    Returns the stream's byte count; raises HQError(HQ_E_STATE) when `out` cannot hold it (the
    encoder wants HQ_EVENT_STREAM_MAX bytes free before each event)."""
    n = len(offsets) - 1
    assert offsets.dtype == np.uint64 and events.dtype == EVENT_DTYPE
    assert out.dtype == np.uint8 and sizes.dtype == np.uint32 and len(sizes) >= n
    assert offsets.flags.c_contiguous and events.flags.c_contiguous and out.flags.c_contiguous
    nb = ctypes.c_uint64(0)
    _chk(lib.hq_events_encode_sized(n, _p(offsets), _p(events) if len(events) else None,
                                    _p(out), len(out), _p(sizes), ctypes.byref(nb)),
         "hq_events_encode_sized")
    return nb.value


def decode_events(offsets, boffsets, data):
    """hq_events_decode: the rows of an event stream (fields it does not carry are 0)."""
    offsets = np.ascontiguousarray(offsets, np.uint64)
    boffsets = np.ascontiguousarray(boffsets, np.uint64)
    data = np.ascontiguousarray(data, np.uint8)
    n = len(offsets) - 1
    ev = np.zeros(max(1, int(offsets[-1]) if n > 0 else 0), EVENT_DTYPE)
    _chk(lib.hq_events_decode(n, _p(offsets), _p(boffsets),
                              _p(data) if len(data) else _p(np.zeros(1, np.uint8)), _p(ev)),
         "hq_events_decode")
    return ev[:int(offsets[-1]) if n > 0 else 0]


# ------------------------------------------------------------------------------ wire decode ----
def decode_batch(data: bytes):
    """hq_wire_decode_batch: (WIRE_MESSAGE_DTYPE array, WireBatchInfo) of one MessageBatch."""
    buf = np.frombuffer(data, np.uint8) if len(data) else np.zeros(1, np.uint8)
    n = ctypes.c_uint64(0)
    info = WireBatchInfo()
    _chk(lib.hq_wire_decode_batch(_p(buf), len(data), None, 0, ctypes.byref(n),
                                  ctypes.byref(info)), "hq_wire_decode_batch")
    out = np.zeros(max(1, n.value), WIRE_MESSAGE_DTYPE)
    _chk(lib.hq_wire_decode_batch(_p(buf), len(data), _p(out), n.value, ctypes.byref(n),
                                  ctypes.byref(info)), "hq_wire_decode_batch")
    return out[:n.value], info


def encode_wire_batch(msgs, deployment_id=0, source_address=b"", out=None):
    """hq_wire_encode_batch: one MessageBatch of WIRE_MESSAGE_DTYPE messages (no entries), as
    the sending node marshals it. Into `out` (uint8, e.g. pinned) when given: returns the bytes
    written as a view of it; else a new array."""
    m = np.ascontiguousarray(msgs, WIRE_MESSAGE_DTYPE)
    src = np.frombuffer(source_address, np.uint8) if source_address else np.zeros(1, np.uint8)
    if out is None:
        out = np.empty(len(m) * 160 + len(source_address) + 24, np.uint8)
    n = ctypes.c_uint64(0)
    _chk(lib.hq_wire_encode_batch(_p(m) if len(m) else None, len(m), deployment_id, _p(src),
                                  len(source_address), _p(out), len(out), ctypes.byref(n)),
         "hq_wire_encode_batch")
    return out[:n.value]


class Wire:
    """hq_wire: a step's input assembled from received MessageBatch bytes and local events."""

    def __init__(self, deployment_id: int = 0):
        self.h = _vp()
        _chk(lib.hq_wire_open(deployment_id, ctypes.byref(self.h)), "hq_wire_open")
        self._inp = StepInput()

    def close(self) -> None:
        if self.h:
            lib.hq_wire_close(self.h)
            self.h = None

    def _check(self, rc: int, what: str) -> None:
        if rc != HQ_OK:
            raise HQError(rc, f"{what}: {lib.hq_wire_last_error(self.h).decode()}")

    def reset(self) -> None:
        self._check(lib.hq_wire_reset(self.h), "hq_wire_reset")

    def add_local(self, cluster_id: int, events: np.ndarray) -> None:
        ev = np.ascontiguousarray(events, EVENT_DTYPE)
        self._check(lib.hq_wire_add_local(self.h, cluster_id, _p(ev), len(ev)),
                    "hq_wire_add_local")

    def add_batch(self, data: bytes) -> None:
        buf = np.frombuffer(data, np.uint8) if len(data) else np.zeros(1, np.uint8)
        self._check(lib.hq_wire_add_batch(self.h, _p(buf), len(data)), "hq_wire_add_batch")

    def add_batch_at(self, addr: int, n: int) -> None:
        """hq_wire_add_batch of n bytes at a raw address (a prepared buffer; no copy)."""
        self._check(lib.hq_wire_add_batch(self.h, _vp(addr), n), "hq_wire_add_batch")

    def add_locals(self, cluster_ids, offsets, events) -> None:
        """hq_wire_add_locals: cluster c's local events are events[offsets[c]:offsets[c + 1]]."""
        c = np.ascontiguousarray(cluster_ids, np.uint64)
        o = np.ascontiguousarray(offsets, np.uint64)
        e = np.ascontiguousarray(events, EVENT_DTYPE)
        assert len(o) == len(c) + 1
        self._check(lib.hq_wire_add_locals(self.h, len(c), _p(c), _p(o), _p(e) if len(e) else None),
                    "hq_wire_add_locals")

    def attach(self, worker: "Worker") -> None:
        """hq_wire_attach: messages resolved to the worker's handles as they are decoded."""
        self._check(lib.hq_wire_attach(self.h, worker.h if worker else None), "hq_wire_attach")

    def step_sized(self, data: np.ndarray, sizes16: np.ndarray):
        """hq_wire_step_sized into the caller's buffers (uint8 `data`, uint16 `sizes16`, e.g.
        pinned): returns (SizedStream over them, WireStats)."""
        assert data.dtype == np.uint8 and sizes16.dtype == np.uint16
        st, out = WireStats(), StepStream()
        self._check(lib.hq_wire_step_sized(self.h, _p(data), len(data), _p(sizes16), len(sizes16),
                                           ctypes.byref(out), ctypes.byref(st)),
                    "hq_wire_step_sized")
        n = out.n_groups
        return SizedStream(None, sizes16[:n], out.n_events, data[:out.n_bytes]), st

    def step_input(self, worker: "Worker"):
        """(groups, offsets, events) numpy views of the assembled hq_step_input (owned by the
        Wire until its next reset), and the WireStats."""
        st = WireStats()
        self._check(lib.hq_wire_step_input(self.h, worker.h, ctypes.byref(self._inp),
                                           ctypes.byref(st)), "hq_wire_step_input")
        n = self._inp.n_groups
        grp = np.ctypeslib.as_array((ctypes.c_uint32 * max(1, n)).from_address(self._inp.groups))[:n] \
            if n else np.zeros(0, np.uint32)
        off = np.ctypeslib.as_array((ctypes.c_uint64 * (n + 1)).from_address(self._inp.offsets))
        ne = int(off[-1]) if n else 0
        ev = np.frombuffer((ctypes.c_char * (ne * EVENT_DTYPE.itemsize)).from_address(
            self._inp.events), EVENT_DTYPE) if ne else np.zeros(0, EVENT_DTYPE)
        return grp.copy(), off.copy(), ev.copy(), st

    def step_stream(self, worker: "Worker"):
        """(groups, offsets, boffsets, bytes) copies of hq_wire_step_stream's output, and the
        WireStats."""
        st = WireStats()
        inp = StepStream()
        self._check(lib.hq_wire_step_stream(self.h, worker.h, ctypes.byref(inp),
                                            ctypes.byref(st)), "hq_wire_step_stream")
        n = inp.n_groups
        grp = np.ctypeslib.as_array((ctypes.c_uint32 * max(1, n)).from_address(inp.groups))[:n] \
            if n else np.zeros(0, np.uint32)
        off = np.ctypeslib.as_array((ctypes.c_uint64 * (n + 1)).from_address(inp.offsets))
        boff = np.ctypeslib.as_array((ctypes.c_uint64 * (n + 1)).from_address(inp.boffsets))
        nb = int(boff[-1]) if n else 0
        data = np.frombuffer((ctypes.c_char * nb).from_address(inp.bytes), np.uint8) if nb \
            else np.zeros(0, np.uint8)
        return grp.copy(), off.copy(), boff.copy(), data.copy(), st
