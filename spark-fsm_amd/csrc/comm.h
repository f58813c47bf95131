// comm.h — collectives of the sharded SPADE path (see comm.cpp).
#pragma once

#include <memory>

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

std::unique_ptr<Comm> make_comm(const fsm_opts& o);
void rccl_unique_id(uint8_t out[128]);

// Longest-processing-time assignment of `n` work units with estimated volumes
// to `nranks` ranks (largest first, ties by index, to the least-loaded rank,
// ties by rank): deterministic, so every rank computes the same plan with no
// communication.  owner[i] = rank of unit i.
void shard_plan(const uint64_t* volume, int64_t n, int32_t nranks, int32_t* owner);

}  // namespace fsm
