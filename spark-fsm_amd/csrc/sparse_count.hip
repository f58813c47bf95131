// sparse_count.hip — the sort half of SPADE's sparse class count (spade_engine.hip,
// Miner::sparse_count): the successful joins of a class batch arrive as u64 keys
// (member slot << 32 | counter column); a radix sort (rocPRIM, LSD over the key
// bits in use) and a run-length encode turn them into the non-zero counters in
// (member slot, column) order, so a batch whose dense D x D counter matrices would
// not fit HBM (a class with tens of thousands of frequent children) is counted in
// memory proportional to its joins.  Kept in its own translation unit: the rocPRIM
// templates are instantiated once, here.
#include <cstring>

#include <rocprim/device/device_radix_sort.hpp>
#include <rocprim/device/device_run_length_encode.hpp>

#include "device_util.h"

namespace fsm {

void sparse_sort_rle(const uint64_t* keys, uint64_t* sorted, uint64_t n, unsigned end_bit, uint64_t* uniq,
                     uint32_t* counts, uint32_t* nruns, hipStream_t s) {
    if (n >= (uint64_t(1) << 32)) throw Error(FSM_ELIMIT, "SPADE: sparse class count of more than 2^32 joins");
    size_t t_sort = 0, t_rle = 0;
    FSM_HIP(rocprim::radix_sort_keys(nullptr, t_sort, keys, sorted, n, 0u, end_bit, s));
    FSM_HIP(rocprim::run_length_encode(nullptr, t_rle, sorted, unsigned(n), uniq, counts, nruns, s));
    DevBuf tmp(std::max<size_t>(std::max(t_sort, t_rle), 16));
    FSM_HIP(rocprim::radix_sort_keys(tmp.p, t_sort, keys, sorted, n, 0u, end_bit, s));
    FSM_HIP(rocprim::run_length_encode(tmp.p, t_rle, sorted, unsigned(n), uniq, counts, nruns, s));
}

}  // namespace fsm
