// hq_dstep.h — the device step engine of the step worker (hq_worker_open_ex with
// HQ_WORKER_ON_DEVICE), shared between hq_worker.cpp (plain C++, the host side: state mirror,
// validation, outputs) and hq_dstep.hip (the kernels). Internal to libhipquorum.so.
#pragma once

#include <cstdint>

#include "../../include/hipquorum.h"

// device-resident group state: one record per group handle
struct hq_dgroup {
    uint64_t cluster_id, node_id, term, committed, last, term_start;
    uint32_t mem;                     // first member in the member pool
    uint8_t n_members, n_voting, state, granted;
    uint8_t rejected, flags, n_reads, pad0;
    uint32_t pad1;
};
static_assert(sizeof(hq_dgroup) == 64, "one 64-byte record per group");

struct hq_dmember {                   // pool order per group: self, remotes, witnesses, observers
    uint64_t node_id, match;
    uint8_t role, active, order, pad[5];
};
static_assert(sizeof(hq_dmember) == 24, "24-byte member records");

struct hq_dread {                     // a pending ReadIndex (readStatus, readindex.go:21-26)
    uint64_t index, from, low, high;
    uint8_t confirmed, pad[7];        // voting slots that acknowledged it
};
static_assert(sizeof(hq_dread) == 40, "40-byte read records");

constexpr uint32_t kDReads = 8;       // pending ReadIndex ctxs per group
constexpr uint32_t kDMembers = 16;    // members per group on the device path
constexpr uint8_t kDSuspended = 1;

struct hq_dstep;                      // device buffers of one worker

struct hq_wait_clock {                // one wait of a step's thread (host steady clock, ns)
    uint64_t t_begin_ns, t_end_ns;    // the wait's start (all queued) and return
    uint64_t poll_ns, sleep_ns;       // polling, then asleep (blocking event or timed sleeps)
    uint64_t sleeps;                  // the sleeps (HQ_WAIT_SLEEP) or 1 (a blocking wait)
    uint64_t device_end_ticks;        // HQ_WAIT_CLOCK: the device's 100-MHz clock after the step
    uint64_t device_start_ticks;      //   and before its first kernel (the jobs path)
};

struct hq_dstep_out {                 // the lists of one step, in input group order, in the
    const hq_commit_event *commits;   // engine's pinned host buffer (valid until its next step)
    const hq_ready_to_read *ready;    // (NULL when the records are compact)
    const hq_ready_compact *ready_compact;
    const hq_read_index_resp *resps;
    const hq_state_change *states;
    const hq_dropped_read *dropped;
    const uint64_t *deferred;
    const uint64_t *fallback;
    uint64_t n_commits, n_ready, n_resps, n_states, n_dropped, n_deferred, n_fallback;
    uint64_t decisions;
    const uint64_t *commit_col;       // the commits as a column (hq_dstep_open's commit_column
                                      // and more than half of the groups committing), else NULL
    const uint32_t *commit_adv;       // the commits as advances (4 bytes per group), else NULL
    uint32_t input_error;             // HQ_E_INVAL: bit 1 unknown handle, 2 offsets, 4 boffsets,
                                      // 8 a group listed twice (no group state written)
    uint64_t kernel_ns, d2h_ns;       // wall time: H2D + pass A + scan + bases; pass B + D2H
    uint64_t submit_ns;               // host time from the call to the last queued operation
    uint64_t gpu_ns;                  // GPU time from the step's first queued operation on the
                                      // compute stream to its last (HIP events; 0: not timed)
    uint32_t gpu_jobs;                // the jobs whose steps shared those launches (1: its own)
    hq_wait_clock wait;               // the step's thread waiting for the device
    // HQ_WORKER_READY_SLOTS (a step that wrote them; else NULL / 0): tile t's single ReadyToReads
    // at ready_slots[256 t ..], slot_counts[t] of them, n_slotted in all
    const hq_ready_compact *ready_slots;
    const uint32_t *slot_counts;
    uint64_t n_tiles, n_slotted;
};

// one step's input: rows (events), an event stream (bytes + boffsets), or an event stream with
// per-group sizes (sizes + the totals; offsets / boffsets unused: the engine scans the sizes)
struct hq_dstep_in {
    uint64_t n;
    const uint32_t *groups;
    const uint64_t *offsets;
    const hq_event *events;
    const uint64_t *boffsets;
    const uint8_t *bytes;
    const uint32_t *sizes = nullptr;   // per group: events | bytes << 16
    uint64_t n_events = 0, n_bytes = 0;
    const uint16_t *sizes16 = nullptr; // or per group: bytes (the engine counts the events)
};

// commit_column: bit 1 a step may return its commits as a column (HQ_WORKER_COMMIT_COLUMN), bit 2
// as a column of advances (HQ_WORKER_COMMIT_ADVANCE), bit 4 its ReadyToReads as 24-byte records
// (HQ_WORKER_READY_COMPACT), bit 8 the single ReadyToReads in per-tile slots (HQ_WORKER_READY_SLOTS)
int hq_dstep_open(hq_ctx *ctx, hq_dstep **out, uint32_t commit_column = 0);
// the step thread's wait (HQ_WAIT_* of include/hipquorum.h, | HQ_WAIT_CLOCK)
int hq_dstep_set_wait(hq_dstep *d, uint32_t mode, uint32_t poll_us, uint32_t sleep_us);
void hq_dstep_close(hq_dstep *d);
// copy group records [g0, g0 + ng) with their reads (kDReads per group) and member records
// [m0, m0 + nm) to the device, growing the device arrays to hold them
int hq_dstep_put(hq_dstep *d, uint64_t g0, uint64_t ng, const hq_dgroup *g, const hq_dread *r,
                 uint64_t m0, uint64_t nm, const hq_dmember *m);
// copy the first ng group records (with their reads) and nm member records back
int hq_dstep_get(hq_dstep *d, uint64_t ng, hq_dgroup *g, hq_dread *r, uint64_t nm, hq_dmember *m);
// one step over the device state; the kernels check the input (out->input_error)
int hq_dstep_run(hq_dstep *d, const hq_dstep_in *in, hq_dstep_out *out);
// several engines' steps through shared launches (hq_worker_step_jobs): every input a sized
// stream, every engine on ds[0]'s device, count <= 64; each job's result in rcs[j] and outs[j]
// as hq_dstep_run gives it; returns the first failure
int hq_dstep_run_jobs(hq_dstep *const *ds, const hq_dstep_in *ins, hq_dstep_out *outs, int *rcs,
                      uint32_t count);
constexpr uint32_t kDStepMaxJobs = 64;

// hq_worker.cpp, for hq_worker_step_jobs (hq_jobs.cpp): the jobs stepped through shared device
// launches when they allow it; kJobsNotFused (nothing done) when they do not
constexpr int kJobsNotFused = 1 << 30;
int hq_worker_step_jobs_fused(hq_step_job *jobs, uint32_t count);
