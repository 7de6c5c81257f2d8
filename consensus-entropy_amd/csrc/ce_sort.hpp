// ce_sort.hpp -- selections with q beyond the list kernels (q > CE_MAX_Q):
// the reference's full ordering np.argsort(ent)[::-1][:q] (amg_test.py:445,
// :452, :480) for ANY q -- `-q` is any integer (:547-553) and argsort returns
// min(q, N) positions.
//
// Records {order key, position} (Cand, 16 B) are sorted by a stable LSD radix
// sort, 8 bits per pass.  The records are generated in ascending position
// order, so 8 passes over the key (descending: digit 255 - byte) leave equal
// keys in ascending position -- the engine's total order (NaN first, entropy
// descending, lowest position).  Batched users add passes over the user id
// held in the record's high position bits (more significant than the key), so
// every user's items end up contiguous, each in the total order.
//
// A pass is three launches, every wave of the grid owning one contiguous
// chunk of the pass input (its items keep their order):
//   k_sort_hist     per-wave digit counts (one LDS counter per digit, bumped by
//                   the leader of each group of lanes holding one digit: the
//                   groups come from 8 ballots, no LDS atomics);
//   k_sort_scan     per digit, the exclusive prefix over the waves;
//   k_sort_scatter  every wave re-reads its chunk in order; a record goes to
//                   digit base + the wave's prefix + its rank among the lanes
//                   of its digit (popcount of the lower peers) -- stable.
// Memory-bound (16 B read twice + written once per record per pass); this
// path is for q above the list kernels' 2048, not the BASELINE configs (q = 10).
// Keys of excluded items (a session's queried songs) are 0, which no entropy
// maps to: they sort last and read back as padding.
#pragma once
#include "ce_topq.hpp"

namespace ce {

constexpr int kSortMaxWaves = 4096;
constexpr int64_t kSortMinChunk = 1024;  // items per wave at least (16 steps)

// One pass: digit of a record.  field 0: the key, descending; field 1: the
// position bits [shift, shift + 8), ascending.
struct SortPass {
    int field;
    int shift;
};

struct SortGeom {
    int64_t n;      // records
    int64_t chunk;  // records per wave (a multiple of 64)
    int nw;         // waves (= cdiv(n, chunk))
};

// Batched users on the sort path: the record's position holds (user <<
// kUserShift) | user-local position
constexpr int kUserShift = 40;
constexpr int kSortMaxUsers = 1 << 23;

// The sort path's workspace (after the 64 KiB header): entropies, two record
// buffers, the per-wave digit counts, the digit totals, and `extra` records.
struct SortWs {
    double* ent;
    Cand* a;
    Cand* b;
    uint32_t* hist;
    uint64_t* dtot;
    Cand* extra;
    SortGeom g;
};

}  // namespace ce
