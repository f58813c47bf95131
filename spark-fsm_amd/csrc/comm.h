// comm.h — collectives of the sharded SPADE path (see comm.cpp).
#pragma once

#include <memory>
#include <string>

#include "fsm_internal.h"

namespace fsm {

class Comm {
  public:
    Comm(int nranks, int rank) : nranks_(nranks), rank_(rank) {}
    virtual ~Comm() = default;
    int nranks() const { return nranks_; }
    int rank() const { return rank_; }
    // in-place sum over ranks of a device u32 array (stream-ordered)
    virtual void allreduce_u32(uint32_t* dev, size_t n, hipStream_t s) = 0;
    // recv[r * bytes .. (r+1) * bytes) = rank r's send block (device buffers)
    virtual void allgather(const void* dev_send, void* dev_recv, size_t bytes, hipStream_t s) = 0;
    // host-memory forms (synchronous)
    virtual void host_allreduce_u32(uint32_t* h, size_t n, hipStream_t s);
    virtual void host_allgather(const void* send, void* recv, size_t bytes, hipStream_t s);
    // every rank's byte blob, concatenated in rank order; sizes[r] = rank r's length
    std::vector<uint8_t> gather_blobs(const std::vector<uint8_t>& mine, std::vector<size_t>& sizes, hipStream_t s);

  private:
    int nranks_, rank_;
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
    // FSM_INJECT_FAIL="<rank>,<phase>": throw FSM_ELIMIT on that rank at that phase
    // (test hook for the agreement)
    void maybe_inject(const char* phase) const;
};

std::unique_ptr<Comm> make_comm(const fsm_opts& o);
void rccl_unique_id(uint8_t out[128]);

// Longest-processing-time assignment of `n` work units with estimated volumes
// to `nranks` ranks (largest first, ties by index, to the least-loaded rank,
// ties by rank): deterministic, so every rank computes the same plan with no
// communication.  owner[i] = rank of unit i.
void shard_plan(const uint64_t* volume, int64_t n, int32_t nranks, int32_t* owner);

}  // namespace fsm
