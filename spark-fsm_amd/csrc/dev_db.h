// dev_db.h — the flattened DBs resident in HBM (built by fsm_db_from_*: the
// host flatten + upload, or K0 on the device, k0_build.hip).
#pragma once

#include <vector>

#include "fsm_internal.h"

// SPADE: one row per distinct sequence id; each row holds its distinct items
// (ascending dense id) with the W-word mask of their rank-compressed eids.
struct SpadeDevDB {
    fsm::DevBuf row_off;  // u32 [R+1]
    fsm::DevBuf item;     // u32 [E]
    fsm::DevBuf mask;     // u64 [E*W]
    int64_t R = 0, E = 0, U = 0;
    int W = 1;
    // the DB-direct root (spade_engine.hip): offset in row << 16 | row length of every
    // entry, made by the first mine that needs it; pos_state 0 = not made, 1 = made,
    // -1 = a row exceeds 65535 entries (that DB keeps the root slab)
    fsm::DevBuf pos;      // u32 [E]
    int pos_state = 0;
};

// TSR: horizontal rows (sid = row) of (item, first, last itemset index),
// item-sorted; the vertical transpose and sid bitmaps are built on the device.
struct TsrDevDB {
    fsm::DevBuf row_off, item, first, last;  // horizontal
    fsm::DevBuf vert_off, vert_sid, vert_item;
    fsm::DevBuf bm;                          // sid bitmaps: U x NW u32 (empty when over budget)
    int64_t N = 0, E = 0, U = 0;
    uint32_t NW = 0;                         // u32 words per item bitmap = ceil(N / 128) * 4 (16-byte rows)
    std::vector<uint32_t> sup;               // |sids(item)|
};

namespace fsm {
// tsr_engine.hip: vertical transpose + sid bitmaps + supports of a TSR DB whose rows are in HBM
void tsr_finish(fsm_ctx* ctx, TsrDevDB* d);
// k0_build.hip: K0 on the device from the token stream; false = this input takes the host flatten
bool k0_build(fsm_ctx* ctx, int mode, const Source& src, fsm_db* db);
}  // namespace fsm
