// Package hipquorum binds libhipquorum.so (include/hipquorum.h), the MI355X batched quorum
// engine, for dragonboat's step workers. It is the new internal package the integration adds
// (INTEGRATION.md): the quorum arithmetic of internal/raft (raft.tryCommit / sortMatchValues,
// raft.go:861-909; readIndex.confirm, readindex.go:77-116; the vote tally, raft.go:1062-1080 and
// 1968-1985; leaderHasQuorum, raft.go:380-390) decided for every leader group of a step worker
// in one call.
//
// The cgo conventions follow the reference's own RocksDB binding
// (internal/logdb/kv/rocksdb/gorocksdb/db.go:3-9 preamble; errors returned as values, db.go:241-253;
// zero-copy slices over C memory, gorocksdb/util.go:27-40): every buffer the library reads during
// or after a call lives in C memory (pinned host memory from AllocPinned, or device memory from
// AllocDevice), so no Go pointer is retained by C.
//
// This file cannot be compiled in the image the library is built in (no Go toolchain); the C
// calls it makes are checked name by name, argument count by argument count and field by field
// against include/hipquorum.h by tests/test_cgo_binding.py.
package hipquorum

/*
#cgo CFLAGS: -I${SRCDIR}/../../include
#cgo LDFLAGS: -L${SRCDIR}/../../dragonboat_amd/lib -lhipquorum -Wl,-rpath,${SRCDIR}/../../dragonboat_amd/lib
#include <stdlib.h>
#include "hipquorum.h"
*/
import "C"

import (
	"errors"
	"fmt"
	"unsafe"
)

// ErrABI is returned by Open when the loaded library implements another ABI than the header
// this package was built against.
var ErrABI = errors.New("hipquorum: library ABI differs from include/hipquorum.h")

func checkABI() error {
	if got := int(C.hq_abi_version()); got != int(C.HQ_ABI_VERSION) {
		return fmt.Errorf("%w (library %d, header %d)", ErrABI, got, int(C.HQ_ABI_VERSION))
	}
	return nil
}

// DeviceCount is the number of GPUs the library sees.
func DeviceCount() (int, error) {
	if err := checkABI(); err != nil {
		return 0, err
	}
	var n C.int
	if rc := C.hq_device_count(&n); rc != C.HQ_OK {
		return 0, errors.New(C.GoString(C.hq_last_error(nil)))
	}
	return int(n), nil
}

// Ctx is one step worker's handle: one HIP stream on GPU (clusterID % nGPU, partition.go:38).
// Not goroutine-safe, like the step worker that owns it (execengine.go:675-690).
type Ctx struct{ c *C.hq_ctx }

// Open opens a context on GPU device after checking the library's ABI version.
func Open(device int) (*Ctx, error) {
	if err := checkABI(); err != nil {
		return nil, err
	}
	var c *C.hq_ctx
	if rc := C.hq_open(C.int(device), 0, &c); rc != C.HQ_OK {
		return nil, errors.New(C.GoString(C.hq_last_error(nil)))
	}
	return &Ctx{c: c}, nil
}

// Close waits for the context's stream and frees it.
func (x *Ctx) Close() {
	C.hq_close(x.c)
	x.c = nil
}

func (x *Ctx) err(rc C.int) error {
	if rc == C.HQ_OK {
		return nil
	}
	return fmt.Errorf("hipquorum error %d: %s", int(rc), C.GoString(C.hq_last_error(x.c)))
}

// Sync waits for every call queued on the context.
func (x *Ctx) Sync() error { return x.err(C.hq_sync(x.c)) }

// WaitFor orders this context's later calls after everything queued on other so far.
func (x *Ctx) WaitFor(other *Ctx) error { return x.err(C.hq_wait_for(x.c, other.c)) }

// AllocPinned allocates pinned host memory the GPU reads and writes directly.
func (x *Ctx) AllocPinned(bytes int) (unsafe.Pointer, error) {
	var p unsafe.Pointer
	if rc := C.hq_alloc_pinned(x.c, C.size_t(bytes), &p); rc != C.HQ_OK {
		return nil, x.err(rc)
	}
	return p, nil
}

// FreePinned frees memory from AllocPinned.
func (x *Ctx) FreePinned(p unsafe.Pointer) error { return x.err(C.hq_free_pinned(x.c, p)) }

// AllocDevice allocates device memory (HBM) on the context's GPU.
func (x *Ctx) AllocDevice(bytes int) (unsafe.Pointer, error) {
	var p unsafe.Pointer
	if rc := C.hq_malloc_dev(x.c, C.size_t(bytes), &p); rc != C.HQ_OK {
		return nil, x.err(rc)
	}
	return p, nil
}

// FreeDevice frees memory from AllocDevice.
func (x *Ctx) FreeDevice(p unsafe.Pointer) error { return x.err(C.hq_free_dev(x.c, p)) }

// CopyAsync queues a copy on the context's stream (kind: 1 host to device, 2 device to host,
// 3 device to device, as hipMemcpyKind).
func (x *Ctx) CopyAsync(dst, src unsafe.Pointer, bytes, kind int) error {
	return x.err(C.hq_memcpy_async(x.c, dst, src, C.size_t(bytes), C.int(kind)))
}

// PinnedU64 views n words of pinned memory as a Go slice (no copy).
func PinnedU64(p unsafe.Pointer, n int) []uint64 { return unsafe.Slice((*uint64)(p), n) }

// PinnedU16 views n halfwords of pinned memory as a Go slice (no copy).
func PinnedU16(p unsafe.Pointer, n int) []uint16 { return unsafe.Slice((*uint16)(p), n) }

// PinnedU8 views n bytes of pinned memory as a Go slice (no copy).
func PinnedU8(p unsafe.Pointer, n int) []uint8 { return unsafe.Slice((*uint8)(p), n) }

// CommitBatch is the structure-of-arrays view of one step's leader groups (DESIGN.md §2), all
// slices over pinned C memory: Match[s*G + g] is voting slot s of group g (the leader, then its
// remotes, then its witnesses; observers are never packed, raft.go:888-909).
type CommitBatch struct {
	G, NMax           int
	Match             []uint64
	NVoting           []uint8 // optional: per-group voter count (nil: every group has NMax)
	Committed, Last   []uint64
	TermMask          []uint16 // bit (i mod 16) = term(i) == r.term for i in (last - 16, last]
	Changed, Fallback []uint64 // ceil(G/64) words each
}

func ptrU64(s []uint64) *C.uint64_t {
	if len(s) == 0 {
		return nil
	}
	return (*C.uint64_t)(unsafe.Pointer(&s[0]))
}

func ptrU16(s []uint16) *C.uint16_t {
	if len(s) == 0 {
		return nil
	}
	return (*C.uint16_t)(unsafe.Pointer(&s[0]))
}

func ptrU8(s []uint8) *C.uint8_t {
	if len(s) == 0 {
		return nil
	}
	return (*C.uint8_t)(unsafe.Pointer(&s[0]))
}

// args is the batch as hq_commit_args in the term-mask form over columns; committed is decided
// in place (commitTo semantics, logentry.go:323-332).
func (b *CommitBatch) args() C.hq_commit_args {
	return C.hq_commit_args{
		G:             C.uint64_t(b.G),
		n_max:         C.uint32_t(b.NMax),
		form:          C.HQ_FORM_TERM_MASK,
		ring_len:      16,
		layout:        C.HQ_LAYOUT_COLUMNS,
		match_stride:  C.uint64_t(b.G),
		match:         ptrU64(b.Match),
		n_voting:      ptrU8(b.NVoting),
		committed_in:  ptrU64(b.Committed),
		committed_out: ptrU64(b.Committed),
		last_index:    ptrU64(b.Last),
		changed:       ptrU64(b.Changed),
		fallback:      ptrU64(b.Fallback),
		term_mask:     ptrU16(b.TermMask),
	}
}

// Commit decides the batch (hq_commit: host pointers staged through the context's device
// workspace), synchronously. Groups whose Changed bit is set commit Committed[g]; groups whose
// Fallback bit is set go through raft.tryCommit on the CPU.
func (x *Ctx) Commit(b *CommitBatch) error {
	a := b.args()
	return x.err(C.hq_commit(x.c, &a))
}

// TileBatch is a batch resident in device memory as leader-row tiles (the headline layout,
// HQ_LAYOUT_TILES_LEADER), e.g. a step worker's device-resident progress table.
type TileBatch struct {
	G, NMax          int
	Tiles            unsafe.Pointer // device: hq_commit_tile_words_for(NMax, mask, layout) words per 128 groups
	CommittedOut     unsafe.Pointer // device [G], or nil with InPlace
	Changed          unsafe.Pointer // device [ceil(G/64)]
	Fallback         unsafe.Pointer // device [ceil(G/64)] or nil
	InPlace          bool           // decide into the table's committed row (HQ_LAYOUT_IN_PLACE)
}

// Args is the batch as the C call takes it.
func (t *TileBatch) Args() C.hq_commit_args {
	layout := C.uint32_t(C.HQ_LAYOUT_TILES_LEADER)
	if t.InPlace {
		layout |= C.HQ_LAYOUT_IN_PLACE
	}
	return C.hq_commit_args{
		G:             C.uint64_t(t.G),
		n_max:         C.uint32_t(t.NMax),
		form:          C.HQ_FORM_TERM_MASK,
		ring_len:      16,
		layout:        layout,
		match:         (*C.uint64_t)(t.Tiles),
		committed_out: (*C.uint64_t)(t.CommittedOut),
		changed:       (*C.uint64_t)(t.Changed),
		fallback:      (*C.uint64_t)(t.Fallback),
	}
}

// TileWords is the size of one 128-group tile in u64 words.
func TileWords(nMax int) int {
	return int(C.hq_commit_tile_words_for(C.uint32_t(nMax), C.HQ_FORM_TERM_MASK,
		C.HQ_LAYOUT_TILES_LEADER))
}

// CommitDev queues the decision of a device-resident batch on the context's stream.
func (x *Ctx) CommitDev(t *TileBatch) error {
	a := t.Args()
	return x.err(C.hq_commit_dev(x.c, &a))
}

// CommitFused decides up to 32 device batches (several step workers' batches of a step, or one
// worker's voter-count buckets) in one launch.
func (x *Ctx) CommitFused(ts []*TileBatch) error {
	if len(ts) == 0 {
		return nil
	}
	n := len(ts)
	mem := C.malloc(C.size_t(n) * C.size_t(unsafe.Sizeof(C.hq_commit_args{})))
	defer C.free(mem)
	as := unsafe.Slice((*C.hq_commit_args)(mem), n)
	for i, t := range ts {
		as[i] = t.Args()
	}
	return x.err(C.hq_commit_fused_dev(x.c, &as[0], C.uint32_t(n)))
}

// LagBatch is one step's leader groups as int32 distances below lastIndex (DESIGN.md §2), device
// columns packed by PackLags from pinned host columns.
type LagBatch struct {
	dev C.hq_commit_lag_args
}

// PackLags packs host columns (Match [NMax][G], Committed, Last, TermMask) into the lag columns
// named by the device argument block (the packer reads lastIndex anyway).
func PackLags(b *CommitBatch, out *LagBatch) error {
	if rc := C.hq_pack_lags(C.uint64_t(b.G), C.uint32_t(b.NMax), ptrU64(b.Match), C.uint64_t(b.G),
		ptrU64(b.Committed), ptrU64(b.Last), nil, ptrU16(b.TermMask), &out.dev); rc != C.HQ_OK {
		return fmt.Errorf("hq_pack_lags: %d", int(rc))
	}
	return nil
}

// CommitLag decides the lag batch and unpacks the decided lags into committed indexes with
// commitTo semantics (logentry.go:323-332).
func (x *Ctx) CommitLag(b *LagBatch, last, fallback, committed []uint64, coutLag []int32) error {
	if err := x.err(C.hq_commit_lag_dev(x.c, &b.dev)); err != nil {
		return err
	}
	if err := x.Sync(); err != nil {
		return err
	}
	if rc := C.hq_unpack_lags(C.uint64_t(len(last)), ptrU64(last),
		(*C.int32_t)(unsafe.Pointer(&coutLag[0])), ptrU64(fallback), ptrU64(committed)); rc != C.HQ_OK {
		return fmt.Errorf("hq_unpack_lags: %d", int(rc))
	}
	return nil
}

// ReadIndexRelease is one step's leader groups with pending ReadIndex ctxs: tiles built by
// hq_tile_ri_multi_dev (device), the compact outputs Count / End in pinned memory, CtxIndex on
// the host as [KMax][G] (non-decreasing per group, addRequest, readindex.go:43-67).
type ReadIndexRelease struct {
	G, KMax, NMax int
	Tiles         unsafe.Pointer // device
	CtxIndex      []uint64
	Count, End    []uint8 // released prefix length and batch-end bits per group (pinned)
	Fallback      []uint64
}

// Decide queues the release (readIndex.confirm, readindex.go:77-116) in its compact form: the
// device writes only Count and End; Released derives each released entry's index.
func (x *Ctx) ReleaseReads(r *ReadIndexRelease) error {
	return x.err(C.hq_readindex_multi_tiles_dev(x.c, C.uint64_t(r.G), C.uint32_t(r.KMax),
		C.uint32_t(r.NMax), (*C.uint8_t)(r.Tiles), 0, C.uint32_t(r.NMax), nil, ptrU8(r.Count),
		ptrU8(r.End), ptrU64(r.Fallback)))
}

// Released calls fn(g, k, index, closer) for every released entry: its read index is the
// index of the ctx that closed its batch (readindex.go:96-104), and the ReadIndexResp messages
// carry that ctx as their hint (raft.go:1740-1760).
func (r *ReadIndexRelease) Released(fn func(g, k int, index uint64, closer int)) {
	for g := 0; g < r.G; g++ {
		closer := -1
		for k := r.KMax - 1; k >= 0; k-- {
			if r.End[g]>>uint(k)&1 != 0 {
				closer = k
			}
			if k < int(r.Count[g]) {
				fn(g, k, r.CtxIndex[closer*r.G+g], closer)
			}
		}
	}
}

// QuorumPlanes is a step's ReadIndex acks, votes and CheckQuorum active flags as bit planes in
// device memory (hq_tile_planes_dev / hq_tile_cq_planes_dev), with the bitmap outputs.
type QuorumPlanes struct {
	G                              int
	Planes, ActivePlanes           unsafe.Pointer // device
	Confirmed, Outcome, HasQuorum  unsafe.Pointer // device bitmaps / 2-bit codes
}

// Decide queues ReadIndex (readindex.go:84), the vote tally (raft.go:1062-1080, 1968-1985) and
// CheckQuorum (raft.go:380-390, the active flags reset as setNotActive, remote.go:196-198) in
// one pass over the planes.
func (x *Ctx) DecideQuorumPlanes(q *QuorumPlanes) error {
	return x.err(C.hq_readindex_vote_cq_planes_dev(x.c, C.uint64_t(q.G), (*C.uint8_t)(q.Planes),
		(*C.uint8_t)(q.ActivePlanes), (*C.uint64_t)(q.Confirmed), (*C.uint64_t)(q.Outcome),
		(*C.uint64_t)(q.HasQuorum)))
}
