"""The MessageBatch decoder (hq_wire_decode_batch, dragonboat_amd/csrc/hq_wire.cpp; host code, no
GPU) against the hand-derived byte fixtures of tests/golden/wire_fixtures.json (raft.proto
:154-196 as raft.pb.go marshals it), round trips through the restated gogo encoder
(tests/wire_encode.py), any-order / unknown-field inputs and malformed batches. Parity against
Go itself is unpinned (no Go toolchain in this image); the fixtures pin the proto2 wire format."""
import json
import os

import numpy as np
import pytest

import wire_encode as we

FIX = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "wire_fixtures.json")))
FIELDS = ("type", "to", "from", "cluster_id", "term", "log_term", "log_index", "commit", "reject",
          "hint", "hint_high", "n_entries", "has_snapshot")


def as_dict(m):
    ev = m["ev"]
    d = {"type": ev["type"], "from": ev["from"], "term": ev["term"], "log_index": ev["log_index"],
         "reject": ev["reject"], "hint": ev["hint"], "hint_high": ev["hint_high"]}
    for k in ("to", "cluster_id", "log_term", "commit", "n_entries", "has_snapshot"):
        d[k] = m[k]
    assert ev["kind"] == 2   # HQ_EV_MESSAGE
    return {k: int(d[k]) for k in FIELDS}


@pytest.mark.parametrize("fx", FIX["batches"], ids=[b["name"] for b in FIX["batches"]])
def test_hand_built_fixtures(hq, fx):
    msgs, info = hq.decode_batch(bytes.fromhex(fx["hex"]))
    assert [as_dict(m) for m in msgs] == fx["messages"]
    assert info.n_messages == len(fx["messages"])
    assert info.deployment_id == fx["deployment_id"] and info.bin_ver == fx["bin_ver"]
    assert info.source_address_len == fx["source_address_len"]


def test_encoder_matches_the_fixtures():
    """The restated gogo encoder reproduces the hand-derived bytes (so the round trips below
    exercise the reference's layout)."""
    for pin in FIX["gogo_encoder_pins"]:
        b = pin["batch"]
        got = we.batch([we.message(**pin["message"])], b["deployment_id"],
                       b["source_address"].encode(), b["bin_ver"])
        want = next(x["hex"] for x in FIX["batches"] if x["name"] == pin["batch_fixture"])
        assert got.hex() == want


@pytest.mark.parametrize("fx", FIX["malformed"], ids=[b["name"] for b in FIX["malformed"]])
def test_malformed_batches_are_rejected(hq, fx):
    with pytest.raises(hq.HQError):
        hq.decode_batch(bytes.fromhex(fx["hex"]))


def test_round_trip_random_messages(hq):
    rng = np.random.default_rng(7)
    big = [0, 1, 127, 128, 300, (1 << 32) - 1, 1 << 32, (1 << 63) + 5, (1 << 64) - 1]
    want, wire = [], []
    for i in range(500):
        v = lambda: big[int(rng.integers(len(big)))] if rng.random() < 0.3 else int(rng.integers(0, 1 << 40))
        m = dict(type=int(rng.integers(0, 26)), to=v(), frm=v(), cluster_id=v(), term=v(),
                 log_term=v(), log_index=v(), commit=v(), reject=bool(rng.random() < 0.5),
                 hint=v(), hint_high=v())
        ne = int(rng.integers(0, 3))
        ents = [we.entry(v(), v(), bytes(rng.integers(0, 256, int(rng.integers(0, 40)),
                                                      dtype=np.uint8))) for _ in range(ne)]
        wire.append(we.message(**m, entries=ents))
        want.append({"type": m["type"], "to": m["to"], "from": m["frm"],
                     "cluster_id": m["cluster_id"], "term": m["term"], "log_term": m["log_term"],
                     "log_index": m["log_index"], "commit": m["commit"],
                     "reject": int(m["reject"]), "hint": m["hint"], "hint_high": m["hint_high"],
                     "n_entries": ne, "has_snapshot": 1})
    msgs, info = hq.decode_batch(we.batch(wire, deployment_id=(1 << 64) - 1,
                                          source_address=b"10.0.0.1:26000"))
    assert [as_dict(m) for m in msgs] == want
    assert info.deployment_id == (1 << 64) - 1 and info.source_address_len == 14


def test_empty_and_header_only_batches(hq):
    msgs, info = hq.decode_batch(b"")
    assert len(msgs) == 0 and info.bin_ver == 0
    msgs, info = hq.decode_batch(we.batch([], deployment_id=5))
    assert len(msgs) == 0 and info.deployment_id == 5 and info.bin_ver == 210


def test_message_with_only_defaults(hq):
    """A proto2 message with every field absent decodes to zeros (a minimal valid encoding)."""
    msgs, _ = hq.decode_batch(we.f_bytes(1, b""))
    assert as_dict(msgs[0]) == {k: 0 for k in FIELDS}


def test_cap_too_small_is_reported(hq):
    import ctypes

    data = we.batch([we.message(type=13, cluster_id=1)] * 3)
    buf = np.frombuffer(data, np.uint8)
    out = np.zeros(2, hq.WIRE_MESSAGE_DTYPE)
    n = ctypes.c_uint64(0)
    rc = hq.lib.hq_wire_decode_batch(hq._p(buf), len(data), hq._p(out), 2, ctypes.byref(n), None)
    assert rc == hq.HQ_E_STATE and n.value == 3


def test_encode_batch_matches_the_marshaller(hq):
    """hq_wire_encode_batch (the sending node's MessageBatch.MarshalTo, bench infrastructure)
    writes exactly the bytes of the Python restatement (tests/wire_encode.py, pinned by the
    hand-derived fixtures), for messages with small and 10-byte varints; they decode back."""
    rng = np.random.default_rng(21)
    n = 300
    m = np.zeros(n, hq.WIRE_MESSAGE_DTYPE)
    big = lambda k: rng.integers(0, 1 << 63, k, dtype=np.uint64) * np.uint64(2) + \
        rng.integers(0, 2, k, dtype=np.uint64)
    for f in ("from", "term", "log_index", "hint", "hint_high"):
        m["ev"][f] = np.where(rng.random(n) < 0.5, rng.integers(0, 300, n).astype(np.uint64), big(n))
    m["ev"]["type"] = rng.integers(0, 30, n)
    m["ev"]["reject"] = rng.integers(0, 2, n)
    m["ev"]["kind"] = hq.EV_MESSAGE
    for f in ("cluster_id", "to", "log_term", "commit"):
        m[f] = np.where(rng.random(n) < 0.5, rng.integers(0, 300, n).astype(np.uint64), big(n))
    got = hq.encode_wire_batch(m, deployment_id=77, source_address=b"n9:1")
    want = we.batch([we.message(type=int(x["ev"]["type"]), to=int(x["to"]), frm=int(x["ev"]["from"]),
                                cluster_id=int(x["cluster_id"]), term=int(x["ev"]["term"]),
                                log_term=int(x["log_term"]), log_index=int(x["ev"]["log_index"]),
                                commit=int(x["commit"]), reject=bool(x["ev"]["reject"]),
                                hint=int(x["ev"]["hint"]), hint_high=int(x["ev"]["hint_high"]))
                     for x in m], deployment_id=77, source_address=b"n9:1")
    assert bytes(got) == want
    dec, info = hq.decode_batch(bytes(got))
    assert info.deployment_id == 77 and len(dec) == n
    for f in ("cluster_id", "to", "log_term", "commit"):
        np.testing.assert_array_equal(dec[f], m[f])
    for f in ("type", "from", "term", "log_index", "hint", "hint_high", "reject"):
        np.testing.assert_array_equal(dec["ev"][f], m["ev"][f])
    with pytest.raises(hq.HQError):
        hq.encode_wire_batch(m, out=np.zeros(100, np.uint8))
