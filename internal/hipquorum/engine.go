package hipquorum

/*
#include <stdlib.h>
#include "hipquorum.h"
*/
import "C"

import (
	"errors"
	"fmt"
	"unsafe"
)

// Engine is the persistent commit engine of one GPU (hq_engine_*): one resident kernel decides
// every step posted to it, with no launch boundary between steps. The step workers whose
// clusters land on the GPU (clusterID % nGPU, partition.go:38) share it: each posts its step's
// batch as soon as it has it, the way workReady.clusterReady wakes a step worker
// (execengine.go:115-123, 860-882), and waits for its own step. Post and Wait are goroutine-safe.
type Engine struct{ e *C.hq_engine }

// EngineConfig selects the batches an engine serves.
type EngineConfig struct {
	NMax    int  // voting slots of every batch
	InPlace bool // batches are device-resident tables decided in place (every post keeps one G)
	Signal  bool // per-step completion (Wait returns when that step is done)
	Depth   int  // steps in flight (power of two 2..64; 0 = 64)
	IdleUs  int  // polling time without a post before the resident launch ends (0 = 1 ms)
}

// OpenEngine opens the engine on the context's GPU (leader-row tiles, term-mask form).
func (x *Ctx) OpenEngine(c EngineConfig) (*Engine, error) {
	cfg := C.hq_engine_config{
		n_max:    C.uint32_t(c.NMax),
		form:     C.HQ_FORM_TERM_MASK,
		layout:   C.HQ_LAYOUT_TILES_LEADER,
		ring_len: 16,
		depth:    C.uint32_t(c.Depth),
		idle_us:  C.uint32_t(c.IdleUs),
	}
	if c.InPlace {
		cfg.layout |= C.HQ_LAYOUT_IN_PLACE
	}
	if c.Signal {
		cfg.flags = C.HQ_ENGINE_SIGNAL
	}
	var e *C.hq_engine
	if rc := C.hq_engine_open(x.c, &cfg, &e); rc != C.HQ_OK {
		return nil, x.err(rc)
	}
	return &Engine{e: e}, nil
}

func (g *Engine) err(rc C.int) error {
	if rc == C.HQ_OK {
		return nil
	}
	return fmt.Errorf("hipquorum engine error %d: %s", int(rc), C.GoString(C.hq_engine_last_error(g.e)))
}

// Post posts one step's batch; it returns the step's sequence number.
func (g *Engine) Post(t *TileBatch) (uint64, error) {
	a := t.Args()
	var seq C.uint64_t
	if rc := C.hq_engine_post(g.e, &a, 1, &seq); rc != C.HQ_OK {
		return 0, g.err(rc)
	}
	return uint64(seq), nil
}

// PostMany posts several steps in order (one call, one lock).
func (g *Engine) PostMany(ts []*TileBatch) (uint64, error) {
	if len(ts) == 0 {
		return 0, errors.New("hipquorum: no batch to post")
	}
	n := len(ts)
	mem := C.malloc(C.size_t(n) * C.size_t(unsafe.Sizeof(C.hq_commit_args{})))
	defer C.free(mem)
	as := unsafe.Slice((*C.hq_commit_args)(mem), n)
	for i, t := range ts {
		as[i] = t.Args()
	}
	var seq C.uint64_t
	if rc := C.hq_engine_post(g.e, &as[0], C.uint32_t(n), &seq); rc != C.HQ_OK {
		return 0, g.err(rc)
	}
	return uint64(seq), nil
}

// Wait returns when step seq is complete: its outputs are in device memory, visible to the
// host and to every stream.
func (g *Engine) Wait(seq uint64) error { return g.err(C.hq_engine_wait(g.e, C.uint64_t(seq))) }

// Step posts a batch and waits for its decisions.
func (g *Engine) Step(t *TileBatch) error {
	seq, err := g.Post(t)
	if err != nil {
		return err
	}
	return g.Wait(seq)
}

// Drain completes every posted step and ends the resident launch (the CUs are free afterwards).
func (g *Engine) Drain() error { return g.err(C.hq_engine_drain(g.e)) }

// Run posts the batches as the next steps and drains: with no launch resident, one launch
// carries the steps and the STOP and ends at the last step (hq_engine_run).
func (g *Engine) Run(ts []*TileBatch) (uint64, error) {
	if len(ts) == 0 {
		return 0, errors.New("hipquorum: no batch to run")
	}
	n := len(ts)
	mem := C.malloc(C.size_t(n) * C.size_t(unsafe.Sizeof(C.hq_commit_args{})))
	defer C.free(mem)
	as := unsafe.Slice((*C.hq_commit_args)(mem), n)
	for i, t := range ts {
		as[i] = t.Args()
	}
	var seq C.uint64_t
	if rc := C.hq_engine_run(g.e, &as[0], C.uint32_t(n), &seq); rc != C.HQ_OK {
		return 0, g.err(rc)
	}
	return uint64(seq), nil
}

// Stats reports the engine's counters.
func (g *Engine) Stats() (posted, completed, relaunches uint64, err error) {
	var s C.hq_engine_stats
	if rc := C.hq_engine_info(g.e, &s); rc != C.HQ_OK {
		return 0, 0, 0, g.err(rc)
	}
	return uint64(s.posted), uint64(s.completed), uint64(s.relaunches), nil
}

// Close drains the engine and frees it.
func (g *Engine) Close() {
	C.hq_engine_close(g.e)
	g.e = nil
}
