// comm.h — collectives of the sharded SPADE path (see comm.cpp).
#pragma once

#include <algorithm>
#include <memory>
#include <string>

#include "fsm_internal.h"

namespace fsm {

struct Agreement;

class Comm {
  public:
    Comm(int nranks, int rank) : nranks_(nranks), rank_(rank) {}
    virtual ~Comm() = default;
    int nranks() const { return nranks_; }
    int rank() const { return rank_; }
    // Work-stealing counters shared by the ranks (not collective): fetch_add returns the
    // counter's previous value (-1: failed).  The RCCL communicator keeps them in a POSIX
    // shared-memory segment of the node, the host communicator calls fsm_host_comm.fetch_add.
    // reset_counter(key) runs on every rank before the collective that precedes the first
    // claim on `key` (the shared-memory slots are reused).  next_key() advances identically
    // on every rank (one key per sharded mine).
    virtual bool has_fetch_add() const { return false; }
    virtual int64_t fetch_add(int64_t /*key*/, int64_t /*inc*/) { return -1; }
    virtual void reset_counter(int64_t /*key*/) {}
    int64_t next_key() { return key_++; }
    int claim_mode = -1;  // agreed over the ranks at the first sharded mine: 1 claims, 0 static plan
    // in-place sum over ranks of a device u32 array (stream-ordered)
    virtual void allreduce_u32(uint32_t* dev, size_t n, hipStream_t s) = 0;
    // recv[r * bytes .. (r+1) * bytes) = rank r's send block (device buffers)
    virtual void allgather(const void* dev_send, void* dev_recv, size_t bytes, hipStream_t s) = 0;
    // host-memory forms (synchronous)
    virtual void host_allreduce_u32(uint32_t* h, size_t n, hipStream_t s);
    virtual void host_allgather(const void* send, void* recv, size_t bytes, hipStream_t s);
    // every rank's byte blob, concatenated in rank order; sizes[r] = rank r's length.
    // agr: the failure agreement rides on the size all-reduce (no round trip of its own):
    // if any rank failed, every rank throws its FSM_E* before the blobs move.  extra[0..n):
    // u32 values summed over the ranks in the same all-reduce.
    // root_only: only rank 0 needs the concatenation (the others may get an empty result;
    // the in-process communicator then copies nothing on them).
    std::vector<uint8_t> gather_blobs(const std::vector<uint8_t>& mine, std::vector<size_t>& sizes, hipStream_t s,
                                      Agreement* agr = nullptr, uint32_t* extra = nullptr, size_t n_extra = 0,
                                      bool root_only = false);

  protected:
    // the blob exchange of gather_blobs once every rank's size is known (sizes[r]):
    // the default pads every blob to the largest and all-gathers them
    virtual std::vector<uint8_t> gather_var(const std::vector<uint8_t>& mine, const std::vector<size_t>& sizes,
                                            hipStream_t s, bool root_only);

  private:
    int nranks_, rank_;
    int64_t key_ = 0;
};

// Failure agreement of a sharded phase: a failure on one rank must not leave
// its peers blocked in a collective.  The work between two collectives runs
// through run(), which records a throw instead of unwinding when there is a
// communicator; agree(), called by every rank before the next collective,
// all-reduces the failure flags and throws the same FSM_E* code on every rank.
struct Agreement {
    Comm* comm = nullptr;
    const char* what = "";  // "SPADE" / "TSR", for the peer message
    int code = 0;
    std::string msg;
    template <class F> void run(F&& f) {
        if (!comm) {
            f();
            return;
        }
        if (code) return;
        try {
            f();
        } catch (const Error& e) {
            code = e.code;
            msg = e.what();
        } catch (const std::bad_alloc&) {
            code = FSM_ENOMEM;
            msg = "host allocation failed";
        } catch (const std::exception& e) {
            code = FSM_EDEVICE;
            msg = e.what();
        }
    }
    void agree(hipStream_t s);
    // flags[c] (c = 1..7) summed over the ranks: throw this rank's failure or a peer's
    void check(const uint32_t* flags) const;
    void flags(uint32_t* f) const {  // this rank's 8 flag slots
        for (int c = 0; c < 8; ++c) f[c] = 0;
        if (code) f[std::clamp(code, 1, 7)] = 1u;
    }
    // FSM_INJECT_FAIL="<rank>,<phase>": throw FSM_ELIMIT on that rank at that phase
    // (test hook for the agreement); FSM_INJECT_STALL (maybe_stall) at the same phases
    void maybe_inject(const char* phase) const;
};

// FSM_INJECT_STALL="<rank>,<phase>,<seconds>": that rank sleeps there (test hook for the
// bounded waits of the in-process group: its peers must return FSM_ECOMM, not hang)
void maybe_stall(int rank, const char* phase);

std::unique_ptr<Comm> make_comm(const fsm_opts& o);
void rccl_unique_id(uint8_t out[128]);
// the limit (ms) of a wait on peer ranks: the environment variable `var` in seconds
// (FSM_COMM_TIMEOUT_S, FSM_COMM_INIT_TIMEOUT_S), default 300 s
double comm_timeout_ms(const char* var);

// In-process ranks: one fsm_ctx driving fsm_opts.ndevices ranks, one host thread
// per rank (fsm_api.cpp, Group).  The ranks' collectives meet in a hub in host
// memory: each rank posts a pointer to its buffer, a barrier, every rank reads the
// others' buffers, a barrier.  Device buffers are staged through host memory (the
// exchanged data are KB-sized: F1 histograms, frequent-pair records, per-launch TSR
// results).  abort() breaks every current and later barrier with FSM_ECOMM, so a
// rank that fails outside a failure agreement cannot leave its peers blocked;
// reset() re-arms the hub once every rank has returned.  A barrier waits at most
// FSM_COMM_TIMEOUT_S for its peers, then aborts the hub and throws FSM_ECOMM (a
// stalled rank never leaves the others blocked without bound).
class InProcHub;
std::shared_ptr<InProcHub> make_inproc_hub(int nranks);
std::unique_ptr<Comm> make_inproc_comm(const std::shared_ptr<InProcHub>& hub, int rank);
void inproc_abort(InProcHub& hub);
bool inproc_aborted(InProcHub& hub);
std::string inproc_state(InProcHub& hub);  // (diagnostics: the group's hang report)
void inproc_reset(InProcHub& hub);

// Longest-processing-time assignment of `n` work units with estimated volumes
// to `nranks` ranks (largest first, ties by index, to the least-loaded rank,
// ties by rank): deterministic, so every rank computes the same plan with no
// communication.  owner[i] = rank of unit i.
void shard_plan(const uint64_t* volume, int64_t n, int32_t nranks, int32_t* owner);

}  // namespace fsm
