package hipquorum

/*
#include <stdlib.h>
#include "hipquorum.h"
*/
import "C"

import (
	"encoding/binary"
	"errors"
	"fmt"
	"runtime"
	"unsafe"

	pb "github.com/lni/dragonboat/v3/raftpb"
)

// Worker is the quorum side of one step worker (hq_worker_*): it takes every quorum-relevant
// event of the worker's nodes for a step — Peer.Handle's filters, handleLeaderReplicateResp,
// handleLeaderHeartbeatResp, handleLeaderReadIndex, handleCandidateRequestVoteResp,
// handleLeaderCheckQuorum, campaign, appendEntries (execengine.go:923-1000 -> node.go:1113-1157)
// — and returns the step's results. One goroutine per worker, like the step worker itself.
type Worker struct {
	w    *C.hq_worker
	rows *C.hq_step_input  // C memory: the argument blocks of the last step
	strm *C.hq_step_stream
	out  *C.hq_step_output
}

func newWorker(w *C.hq_worker) *Worker {
	x := &Worker{w: w}
	x.rows = (*C.hq_step_input)(C.calloc(1, C.size_t(unsafe.Sizeof(C.hq_step_input{}))))
	x.strm = (*C.hq_step_stream)(C.calloc(1, C.size_t(unsafe.Sizeof(C.hq_step_stream{}))))
	x.out = (*C.hq_step_output)(C.calloc(1, C.size_t(unsafe.Sizeof(C.hq_step_output{}))))
	return x
}

// OpenWorker opens a host worker (decisions on the GPU, bookkeeping on the host).
func OpenWorker(device, nMax int) (*Worker, error) {
	if err := checkABI(); err != nil {
		return nil, err
	}
	var w *C.hq_worker
	if rc := C.hq_worker_open(C.int(device), C.uint32_t(nMax), &w); rc != C.HQ_OK {
		return nil, errors.New(C.GoString(C.hq_last_error(nil)))
	}
	return newWorker(w), nil
}

// OpenDeviceWorker opens a worker whose groups' quorum state is resident in HBM: one GPU thread
// per group takes its events in order, every decision at the event that triggers it
// (hq_dstep.hip); commits come back as 4-byte advances when a quarter of the listed groups
// commit, else as one word per listed group or as records; ReadyToReads as 24-byte records
// (EachReady).
func OpenDeviceWorker(device, nMax int) (*Worker, error) {
	if err := checkABI(); err != nil {
		return nil, err
	}
	var w *C.hq_worker
	flags := C.uint32_t(C.HQ_WORKER_ON_DEVICE | C.HQ_WORKER_COMMIT_ADVANCE | C.HQ_WORKER_COMMIT_COLUMN |
		C.HQ_WORKER_READY_COMPACT | C.HQ_WORKER_READY_SLOTS)
	if rc := C.hq_worker_open_ex(C.int(device), C.uint32_t(nMax), flags, &w); rc != C.HQ_OK {
		return nil, errors.New(C.GoString(C.hq_last_error(nil)))
	}
	return newWorker(w), nil
}

func (x *Worker) err(rc C.int) error {
	if rc == C.HQ_OK {
		return nil
	}
	return fmt.Errorf("hipquorum worker error %d: %s", int(rc), C.GoString(C.hq_worker_last_error(x.w)))
}

// Close frees the worker.
// SetWait sets how the worker's goroutine waits for its device step (hq_worker_set_wait:
// C.HQ_WAIT_BLOCK / C.HQ_WAIT_SLEEP / C.HQ_WAIT_SPIN / C.HQ_WAIT_ADAPT, | C.HQ_WAIT_CLOCK).
func (x *Worker) SetWait(mode, pollUs, sleepUs uint32) error {
	return x.err(C.hq_worker_set_wait(x.w, C.uint32_t(mode), C.uint32_t(pollUs), C.uint32_t(sleepUs)))
}

func (x *Worker) Close() {
	C.hq_worker_close(x.w)
	C.free(unsafe.Pointer(x.rows))
	C.free(unsafe.Pointer(x.strm))
	C.free(unsafe.Pointer(x.out))
	x.w = nil
}

// Member is one member of a group as the worker holds it.
type Member = C.hq_member

// GroupState is a group's quorum state (add / set / get).
type GroupState = C.hq_worker_group

// AddGroup registers a group (NodeHost.StartCluster) and returns its handle.
func (x *Worker) AddGroup(g *GroupState, members []Member) (uint32, error) {
	var h C.uint32_t
	var mp *C.hq_member
	if len(members) > 0 {
		mp = &members[0]
	}
	if rc := C.hq_worker_add_group(x.w, g, mp, &h); rc != C.HQ_OK {
		return 0, x.err(rc)
	}
	return uint32(h), nil
}

// SetGroup re-syncs a group after a fallback or a membership change.
func (x *Worker) SetGroup(g *GroupState, members []Member) error {
	var mp *C.hq_member
	if len(members) > 0 {
		mp = &members[0]
	}
	return x.err(C.hq_worker_set_group(x.w, g, mp))
}

// Output is one step's results; the lists live in the worker's pinned buffers and are valid
// until the worker's next step.
type Output struct {
	c      *C.hq_step_output
	listed int
}

// Step hands over the step's events as rows: groups[i]'s events are
// events[offsets[i]:offsets[i+1]] (local ReadIndex, received messages, tick messages, proposals —
// node.handleEvents order). All three slices must be views of pinned C memory.
func (x *Worker) Step(groups []uint32, offsets []uint64, events []C.hq_event) (*Output, error) {
	*x.rows = C.hq_step_input{
		n_groups: C.uint64_t(len(groups)),
		groups:   (*C.uint32_t)(unsafe.Pointer(&groups[0])),
		offsets:  (*C.uint64_t)(unsafe.Pointer(&offsets[0])),
		events:   (*C.hq_event)(unsafe.Pointer(&events[0])),
	}
	if rc := C.hq_worker_step(x.w, x.rows, x.out); rc != C.HQ_OK {
		return nil, x.err(rc)
	}
	return &Output{c: x.out, listed: len(groups)}, nil
}

// StreamBuf is one step's input as an event stream in pinned C memory: per event a header byte
// and the LEB128 varints of the fields its handler reads (include/hipquorum.h "event streams"),
// per node one size word (events | bytes << 16; the sized form of hq_step_stream).
type StreamBuf struct {
	Groups  []uint32 // worker handles, or nil: every handle 0 .. len(Sizes)-1 in order
	Sizes   []uint16 // per node its byte count (hq_step_stream.sizes16: the engine counts events)
	NEvents uint64
	Bytes   []byte // a pinned region; len = bytes written so far
	start   int
	events  int
	prev    prevMsg
}

// the node's stream state the header codes refer back to: its previous message term, its
// previous ReplicateResp's index (code 4), its previous HeartbeatResp's ctx (code 5)
type prevMsg struct {
	term, index, hint, high uint64
	haveIndex               bool
}

// BeginNode starts a node's run of events.
func (b *StreamBuf) BeginNode() {
	b.start = len(b.Bytes)
	b.events = 0
	b.prev = prevMsg{}
}

// EndNode closes the node's run with its size word.
func (b *StreamBuf) EndNode(handle uint32) {
	if b.Groups != nil {
		b.Groups = append(b.Groups, handle)
	}
	b.Sizes = append(b.Sizes, uint16(len(b.Bytes)-b.start))
	b.NEvents += uint64(b.events)
}

func (b *StreamBuf) header(code uint32, reject bool, term uint64) {
	h := byte(C.HQ_EV_MESSAGE) | byte(code<<3)
	if reject {
		h |= 0x40
	}
	same := term == b.prev.term
	if same {
		h |= 0x80
	}
	b.Bytes = append(b.Bytes, h)
	b.prev.term = term
	b.events++
}

// AppendReplicateResp encodes a ReplicateResp (code 0, or code 4 without the index when it
// repeats the node's previous ReplicateResp in this step).
func (b *StreamBuf) AppendReplicateResp(from, term, index uint64, reject bool) {
	code := uint32(0)
	if b.prev.haveIndex && index == b.prev.index {
		code = 4
	}
	b.prev.index, b.prev.haveIndex = index, true
	same := term == b.prev.term
	b.header(code, reject, term)
	b.Bytes = binary.AppendUvarint(b.Bytes, from)
	if !same {
		b.Bytes = binary.AppendUvarint(b.Bytes, term)
	}
	if code == 0 {
		b.Bytes = binary.AppendUvarint(b.Bytes, index)
	}
}

// AppendHeartbeatResp encodes a HeartbeatResp (code 2, or code 5 without the ctx when it repeats
// the node's previous HeartbeatResp ctx; 0 / 0 before the first).
func (b *StreamBuf) AppendHeartbeatResp(from, term uint64, ctx pb.SystemCtx) {
	code := uint32(2)
	if ctx.Low == b.prev.hint && ctx.High == b.prev.high {
		code = 5
	}
	b.prev.hint, b.prev.high = ctx.Low, ctx.High
	same := term == b.prev.term
	b.header(code, false, term)
	b.Bytes = binary.AppendUvarint(b.Bytes, from)
	if !same {
		b.Bytes = binary.AppendUvarint(b.Bytes, term)
	}
	if code == 2 {
		b.Bytes = binary.AppendUvarint(b.Bytes, ctx.Low)
		b.Bytes = binary.AppendUvarint(b.Bytes, ctx.High)
	}
}

// AppendPropose encodes a proposal of n entries (handleLeaderPropose).
func (b *StreamBuf) AppendPropose(n uint64) {
	b.Bytes = append(b.Bytes, byte(C.HQ_EV_PROPOSE))
	b.Bytes = binary.AppendUvarint(b.Bytes, n)
	b.events++
}

// AppendLocalRead encodes the node's own ReadIndex (Peer.ReadIndex, node.go:1197).
func (b *StreamBuf) AppendLocalRead(ctx pb.SystemCtx) {
	b.Bytes = append(b.Bytes, byte(C.HQ_EV_READ))
	b.Bytes = binary.AppendUvarint(b.Bytes, ctx.Low)
	b.Bytes = binary.AppendUvarint(b.Bytes, ctx.High)
	b.events++
}

func (x *Worker) setStream(b *StreamBuf) {
	*x.strm = C.hq_step_stream{
		n_groups: C.uint64_t(len(b.Sizes)),
		bytes:    (*C.uint8_t)(unsafe.Pointer(&b.Bytes[0])),
		sizes16:  (*C.uint16_t)(unsafe.Pointer(&b.Sizes[0])),
		n_events: C.uint64_t(b.NEvents),
		n_bytes:  C.uint64_t(len(b.Bytes)),
	}
	if b.Groups != nil {
		x.strm.groups = (*C.uint32_t)(unsafe.Pointer(&b.Groups[0]))
	}
}

// StepStream steps the worker over an event stream (Bytes, Sizes and Groups in pinned memory).
func (x *Worker) StepStream(b *StreamBuf) (*Output, error) {
	x.setStream(b)
	if rc := C.hq_worker_step_stream(x.w, x.strm, x.out); rc != C.HQ_OK {
		return nil, x.err(rc)
	}
	return &Output{c: x.out, listed: len(b.Sizes)}, nil
}

// StepJobs steps several device workers of one GPU at once through shared launches (the 16
// step-worker goroutines each calling their own worker, execengine.go:923-1000).
func StepJobs(ws []*Worker, bufs []*StreamBuf) ([]*Output, error) {
	n := len(ws)
	if n == 0 || n != len(bufs) {
		return nil, errors.New("hipquorum: one stream per worker")
	}
	mem := C.calloc(C.size_t(n), C.size_t(unsafe.Sizeof(C.hq_step_job{})))
	defer C.free(mem)
	jobs := unsafe.Slice((*C.hq_step_job)(mem), n)
	for i, w := range ws {
		w.setStream(bufs[i])
		jobs[i] = C.hq_step_job{worker: w.w, stream: w.strm, out: w.out}
	}
	rc := C.hq_worker_step_jobs(&jobs[0], C.uint32_t(n))
	outs := make([]*Output, n)
	for i, w := range ws {
		if jobs[i].rc != C.HQ_OK {
			return nil, w.err(jobs[i].rc)
		}
		outs[i] = &Output{c: w.out, listed: len(bufs[i].Sizes)}
	}
	if rc != C.HQ_OK {
		return nil, fmt.Errorf("hq_worker_step_jobs: %d", int(rc))
	}
	return outs, nil
}

// EachCommit calls fn(listed index, new committed index) for every group that committed in the
// step, whichever form the step returned: the advance column (added to the committed index the
// node holds: committedOf), the index column, or the (cluster, index) records (listedOf maps a
// cluster id to its listed index). The node then applies commitTo (logentry.go:323-332).
func (o *Output) EachCommit(committedOf func(i int) uint64, listedOf func(clusterID uint64) int,
	fn func(i int, committed uint64)) {
	switch {
	case o.c.committed_advance != nil:
		adv := unsafe.Slice((*uint32)(unsafe.Pointer(o.c.committed_advance)), o.listed)
		for i, a := range adv {
			if a != 0 {
				fn(i, committedOf(i)+uint64(a))
			}
		}
	case o.c.committed_column != nil:
		col := unsafe.Slice((*uint64)(unsafe.Pointer(o.c.committed_column)), o.listed)
		for i, c := range col {
			if c != 0 {
				fn(i, c)
			}
		}
	default:
		if o.c.n_commits == 0 {
			return
		}
		recs := unsafe.Slice(o.c.commits, int(o.c.n_commits))
		for _, r := range recs {
			fn(listedOf(uint64(r.cluster_id)), uint64(r.committed))
		}
	}
}

// ReadyToRead lists the step's released reads (pb.ReadyToRead, raftpb/raft.go:54-57) when the
// step returned them as full records (nil when they are compact: EachReady reads both).
func (o *Output) ReadyToRead() []C.hq_ready_to_read {
	if o.c.n_ready == 0 || o.c.ready == nil {
		return nil
	}
	return unsafe.Slice(o.c.ready, int(o.c.n_ready))
}

// EachReady calls fn(listed index, pb.ReadyToRead) for every released read of the step, in the
// reference's order (listed order), whichever form the step returned: the per-tile slots
// (HQ_WORKER_READY_SLOTS) and the list — 24-byte records (HQ_WORKER_READY_COMPACT: the index is
// the group's committed index before the step, committedBefore, plus the record's delta) or full
// records (listedOf maps a cluster id to its listed index) — merged by listed index (a group's
// reads are all in one of the two). The node then calls processReadyToRead (node.go:1026-1031).
func (o *Output) EachReady(committedBefore func(i int) uint64, listedOf func(clusterID uint64) int,
	fn func(i int, r pb.ReadyToRead)) {
	compact := func(r C.hq_ready_compact) (int, pb.ReadyToRead) {
		i := int(r.pos)
		return i, pb.ReadyToRead{Index: committedBefore(i) + uint64(int64(r.delta)),
			SystemCtx: pb.SystemCtx{Low: uint64(r.ctx_low), High: uint64(r.ctx_high)}}
	}
	// the list, one record at a time with its listed index
	k, n := 0, int(o.c.n_ready)
	listAt := func(k int) (int, pb.ReadyToRead) {
		if o.c.ready_compact != nil {
			return compact(unsafe.Slice(o.c.ready_compact, n)[k])
		}
		var f C.hq_ready_to_read = unsafe.Slice(o.c.ready, n)[k]
		return listedOf(uint64(f.cluster_id)), pb.ReadyToRead{Index: uint64(f.index),
			SystemCtx: pb.SystemCtx{Low: uint64(f.ctx_low), High: uint64(f.ctx_high)}}
	}
	if o.c.ready_slots != nil {
		tiles := int(o.c.n_ready_tiles)
		counts := unsafe.Slice((*uint32)(unsafe.Pointer(o.c.ready_slot_counts)), tiles)
		slots := unsafe.Slice(o.c.ready_slots, tiles*256)
		for t, c := range counts {
			for _, r := range slots[t*256 : t*256+int(c)] {
				i, rr := compact(r)
				for ; k < n; k++ { // the list's reads of the groups before this one
					j, lr := listAt(k)
					if j > i {
						break
					}
					fn(j, lr)
				}
				fn(i, rr)
			}
		}
	}
	for ; k < n; k++ {
		fn(listAt(k))
	}
}

// StateChanges lists the step's leader / follower / candidate transitions.
func (o *Output) StateChanges() []C.hq_state_change {
	if o.c.n_state_changes == 0 {
		return nil
	}
	return unsafe.Slice(o.c.state_changes, int(o.c.n_state_changes))
}

// FallbackClusters lists the clusters whose later events go through the CPU raft this step.
func (o *Output) FallbackClusters() []uint64 {
	if o.c.n_fallback_groups == 0 {
		return nil
	}
	return unsafe.Slice((*uint64)(unsafe.Pointer(o.c.fallback_groups)), int(o.c.n_fallback_groups))
}

// Msg16 packs one received message for the library's encoder (include/hipquorum.h "Compact
// messages"). A field that does not fit (a node id >= 2^16, a term >= 2^32, a HeartbeatResp ctx
// with a high word that is not the node's own pending read) needs the escape (HQ_EV16_FULL and
// the 56-byte row in 4 records); ok is false then.
func Msg16(m *pb.Message, readCtx pb.SystemCtx) (r C.hq_event16, ok bool) {
	if m.From >= 1<<16 || m.Term >= 1<<32 || uint64(m.Type) >= 256 {
		return r, false
	}
	r = C.hq_event16{kind: C.uint8_t(C.HQ_EV_MESSAGE), _type: C.uint8_t(m.Type),
		from: C.uint16_t(m.From), term: C.uint32_t(m.Term)}
	if m.Reject {
		r.kind |= 8
	}
	switch m.Type {
	case pb.HeartbeatResp, pb.ReadIndex:
		if m.Hint == readCtx.Low && m.HintHigh == readCtx.High && m.Hint|m.HintHigh != 0 {
			r.kind |= C.HQ_EV16_READ_CTX
		} else if m.HintHigh != 0 {
			return r, false
		} else {
			r.value = C.uint64_t(m.Hint)
		}
	default:
		r.value = C.uint64_t(m.LogIndex)
	}
	return r, true
}

// Encode16 encodes a step's compact records (recs[offsets[i]:offsets[i+1]] for listed node i)
// into the stream buffer's bytes and size words on `threads` native threads.
func Encode16(offsets []uint64, recs []C.hq_event16, b *StreamBuf, threads int) error {
	nGroups := len(offsets) - 1
	var nEvents, nBytes C.uint64_t
	var rp *C.hq_event16
	if len(recs) > 0 {
		rp = &recs[0]
	}
	rc := C.hq_events16_encode_sized(C.uint64_t(nGroups), (*C.uint64_t)(unsafe.Pointer(&offsets[0])),
		rp, (*C.uint8_t)(unsafe.Pointer(&b.Bytes[:cap(b.Bytes)][0])), C.uint64_t(cap(b.Bytes)),
		(*C.uint32_t)(unsafe.Pointer(&b.Sizes[:cap(b.Sizes)][0])), &nEvents, &nBytes, C.uint32_t(threads))
	if rc != C.HQ_OK {
		return fmt.Errorf("hq_events16_encode_sized: %d", int(rc))
	}
	b.Bytes = b.Bytes[:int(nBytes)]
	b.Sizes = b.Sizes[:nGroups]
	b.NEvents = uint64(nEvents)
	return nil
}

// Encode16Job is one step worker's step for EncodeMany: its compact records and stream buffer.
type Encode16Job struct {
	Offsets []uint64
	Recs    []C.hq_event16
	Buf     *StreamBuf
}

// EncodeMany encodes the steps of several step workers in one call whose `threads` native
// threads split the records of all of them evenly (hq_events16_encode_sized_multi); each
// buffer ends as its own Encode16 would leave it. The Go slices the C array points at are
// pinned for the call (cgo: Go pointers stored in C memory must be pinned).
func EncodeMany(jobs []Encode16Job, threads int) error {
	if len(jobs) == 0 {
		return nil
	}
	var pin runtime.Pinner
	defer pin.Unpin()
	mem := C.malloc(C.size_t(len(jobs)) * C.size_t(unsafe.Sizeof(C.hq_encode16_job{})))
	defer C.free(mem)
	cj := unsafe.Slice((*C.hq_encode16_job)(mem), len(jobs))
	for i, j := range jobs {
		b := j.Buf
		pin.Pin(&j.Offsets[0])
		bytes := b.Bytes[:cap(b.Bytes)]
		sizes := b.Sizes[:cap(b.Sizes)]
		pin.Pin(&bytes[0])
		pin.Pin(&sizes[0])
		cj[i] = C.hq_encode16_job{n_groups: C.uint64_t(len(j.Offsets) - 1),
			offsets16: (*C.uint64_t)(unsafe.Pointer(&j.Offsets[0])),
			out:       (*C.uint8_t)(unsafe.Pointer(&bytes[0])), cap: C.uint64_t(len(bytes)),
			sizes16: (*C.uint16_t)(unsafe.Pointer(&sizes[0]))}
		if len(j.Recs) > 0 {
			pin.Pin(&j.Recs[0])
			cj[i].recs = &j.Recs[0]
		}
	}
	rc := C.hq_events16_encode_sized_multi(&cj[0], C.uint32_t(len(jobs)), C.uint32_t(threads))
	for i, j := range jobs {
		if cj[i].rc != C.HQ_OK {
			return fmt.Errorf("hq_events16_encode_sized_multi: job %d: %d", i, int(cj[i].rc))
		}
		j.Buf.Bytes = j.Buf.Bytes[:int(cj[i].n_bytes)]
		j.Buf.Sizes = j.Buf.Sizes[:len(j.Offsets)-1]
		j.Buf.NEvents = uint64(cj[i].n_events)
	}
	if rc != C.HQ_OK {
		return fmt.Errorf("hq_events16_encode_sized_multi: %d", int(rc))
	}
	return nil
}
