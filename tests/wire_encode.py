"""Test infrastructure: a restatement of the reference's protobuf marshalling of raftpb.Message and
raftpb.MessageBatch (raftpb/raft.pb.go Message.MarshalTo :2232-2300, MessageBatch.MarshalTo
:2417-2445, Snapshot.MarshalTo :2142, Membership.MarshalTo :2019, Entry.MarshalTo), used to
build MessageBatch bytes for the wire decoder's tests. gogoproto nullable=false fields are
always written, in field-number order, exactly as the generated code does; the byte layout is
pinned by the hand-derived fixtures in tests/golden/wire_fixtures.json."""


def varint(v: int) -> bytes:
    out = bytearray()
    while True:
        b = v & 0x7F
        v >>= 7
        if v:
            out.append(b | 0x80)
        else:
            out.append(b)
            return bytes(out)


def key(field: int, wire: int) -> bytes:
    return varint((field << 3) | wire)


def f_varint(field: int, v: int) -> bytes:
    return key(field, 0) + varint(v)


def f_bytes(field: int, b: bytes) -> bytes:
    return key(field, 2) + varint(len(b)) + b


def membership() -> bytes:
    """An empty Membership: config_change_id = 0, no addresses / removed / observers / witnesses."""
    return f_varint(1, 0)


def snapshot() -> bytes:
    """An empty Snapshot (raft.pb.go:2142): every non-nullable field written, checksum (nullable)
    and files (repeated) omitted."""
    return (f_bytes(2, b"") + f_varint(3, 0) + f_varint(4, 0) + f_varint(5, 0)
            + f_bytes(6, membership()) + f_varint(9, 0) + f_varint(10, 0) + f_varint(11, 0)
            + f_varint(12, 0) + f_varint(13, 0) + f_varint(14, 0))


def entry(term: int, index: int, cmd: bytes = b"") -> bytes:
    """Entry (raft.proto Entry: term 1, index 2, type 3, key 4, client_id 5, series_id 6,
    responded_to 7, cmd 8)."""
    return (f_varint(1, term) + f_varint(2, index) + f_varint(3, 0) + f_varint(4, 0)
            + f_varint(5, 0) + f_varint(6, 0) + f_varint(7, 0) + f_bytes(8, cmd))


def message(type=0, to=0, frm=0, cluster_id=0, term=0, log_term=0, log_index=0, commit=0,
            reject=False, hint=0, entries=(), hint_high=0) -> bytes:
    """Message.MarshalTo (raft.pb.go:2232-2300): fields 1-10, the entries (11), the snapshot (12,
    always), hint_high (13)."""
    b = (f_varint(1, type) + f_varint(2, to) + f_varint(3, frm) + f_varint(4, cluster_id)
         + f_varint(5, term) + f_varint(6, log_term) + f_varint(7, log_index)
         + f_varint(8, commit) + f_varint(9, 1 if reject else 0) + f_varint(10, hint))
    for e in entries:
        b += f_bytes(11, e)
    return b + f_bytes(12, snapshot()) + f_varint(13, hint_high)


def batch(messages, deployment_id=0, source_address=b"", bin_ver=210) -> bytes:
    """MessageBatch.MarshalTo (raft.pb.go:2417-2445)."""
    b = b"".join(f_bytes(1, m) for m in messages)
    return b + f_varint(2, deployment_id) + f_bytes(3, source_address) + f_varint(4, bin_ver)
