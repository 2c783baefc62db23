// common.h — shared host/device definitions of the crdtm engine (gfx950).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <map>
#include <string>
#include <vector>

#include "../../include/crdtm.h"

namespace crdtm {

constexpr uint32_t NONE = 0xFFFFFFFFu;     // absent index / list end
constexpr uint32_t ABSENT = 0xFFFFFFFEu;   // entry not part of a list
constexpr uint32_t PDR_REACHED = 0xFFFFFFFDu;  // K1 tag: the op's path resolved to its leaf dict
constexpr uint32_t TAG_DUP = 0xFFFFFFFAu;      // K1 tag, k_lv_leaf -> k_lv_fin only: an Add whose key is taken (ts 0 or an earlier Add)
constexpr uint32_t TAG_LAZY = 0xFFFFFFFBu;     // K1 tag: stopped at a Tombstone of the chain ending at cur
constexpr uint32_t SENT_T = 0xFFFFFFFDu;       // K1 leaf target: the dict's sentinel (key 0)
constexpr uint32_t MISS_T = 0xFFFFFFFCu;       // K1 leaf target: key not in the dict
constexpr int64_t TWO53 = 9007199254740992LL;
constexpr int64_t TWO32 = 4294967296LL;
constexpr int REPLICA_BITS = 22;           // replica ids in (-2^21, 2^21) when |ts| < 2^53
constexpr uint32_t REPLICA_SLOTS = 1u << REPLICA_BITS;
constexpr int BLOCK = 256;

// Per-op status codes (crdtm.h CRDTM_ST_*) plus internal states.
enum : uint8_t {
  ST_APPLIED = CRDTM_ST_APPLIED,
  ST_ALREADY = CRDTM_ST_ALREADY,
  ST_INVALID = 4,   // Err InvalidPath
  ST_NOTFOUND = 5,  // Err NotFound -> OperationFailed op
  ST_PENDING = 6,
};

// Guard bits (crdtm_result.guard)
enum : uint32_t {
  G_COLLISION = 1u,     // same ts added under two different parents
  G_DEL_BEFORE_ADD = 2u,// a dict saw a Delete before a later Add (tombstones in the skip walk)
  G_REPLICA_DRIFT = 4u, // own replica id changes during the batch (timestamp crosses 2^32)
  G_NOT_FRESH = 8u,     // tree already holds state (incremental merge)
  G_DEEP_PATH = 16u,    // a path longer than the length buckets of K1
  G_FORCED = 32u,       // CRDTM_FORCE_REPLAY=1: the sequential replay on purpose (measures the fallback)
};

// Small device-side result block (one copy back per phase).
constexpr uint32_t REP_INLINE = 256;  // replica entries returned inside the result block

struct DevResult {
  uint32_t err_index;       // atomicMin over erroring ops
  uint32_t guard;           // G_* bits
  uint32_t max_len;         // longest path
  uint32_t bad_range;       // |ts| >= 2^53 present
  uint32_t n_applied;
  uint32_t n_already;
  uint32_t n_adds_applied;
  uint32_t own_ok_adds;     // Ok adds with replicaId(ts) == tree id (timestamp bumps)
  uint32_t n_replica_out;
  uint32_t n_rep_list;      // replicas touched by a commit's fold (k_rep_max)
  uint32_t n_nodes_kept;    // closed form: nodes that survive (dict alive)
  uint32_t n_live_kept;     // kept nodes that own a children dict
  uint32_t n_sentinels;     // present sentinels (Euler)
  uint32_t log_n;           // applied ops (log entries appended)
  uint32_t log_npath;
  uint32_t replay_slots;    // replay: slots used
  uint32_t replay_dicts;
  uint32_t replay_overflow;
  uint32_t replay_err_code;
  int64_t replay_timestamp;
  uint32_t n_split[8];      // list ranking level sizes
  uint32_t big_segments;
  uint32_t huge_segments;
  uint32_t mid_segments;
  uint32_t last_add;        // 1 + index of the last applied Add
  uint32_t first_del;       // index of the first applied Delete
  uint32_t has_negative;    // some Add ts < 0 (dense index impossible)
  uint32_t n_del;           // Delete ops in the batch
  uint32_t range_total;     // dense index size
  uint32_t max_replica;     // largest replica id of an Add timestamp
  uint32_t scan_err;        // a look-back scan gave up (never on a live device)
  uint32_t dup_fix;         // flat status: a duplicate timestamp took its slot, decide again
  uint32_t pdr_conflict;    // per-dict replay: a path crossed a key the copy quirk refilled
  uint32_t pdr_jobs;        // per-dict replay: snapshot dicts created so far
  uint32_t pdr_overflow;    // per-dict replay: snapshot room exhausted
  uint32_t pdr_dicts;       // per-dict replay: dicts of the new state
  uint32_t pdr_slots;       // per-dict replay: slots of the new state
  uint32_t since_end;       // operationsSince: 1 + log index of the newest Add with the asked ts
  // incremental per-dict replay (ilr.hip)
  uint32_t ilr_conflict;    // a case the level replay cannot decide: the batch goes to the re-merge
  uint32_t ilr_overflow;    // slot / dict / undo room exhausted
  uint32_t ilr_slots;       // slot counter (new slots are taken from it)
  uint32_t ilr_dicts;       // dict counter
  uint32_t ilr_undo;        // undo entries used
  uint32_t ilr_groups;      // dict groups of the batch
  uint32_t ilr_why;         // conflict reasons (ilr.hip IW_* bits)
  uint32_t ilr_jobs;        // deferred copies created so far
  // flat claim/check counters, 16 shards one cache line apart (shard k at
  // [32 k]): +0 slots holding an Add, +1 Adds with a timestamp slot, +2 Adds
  // of the own replica, +3 ops that need per-op statuses (empty path, ts 0)
  uint32_t fl_part[16 * 32];
  uint32_t spec_fail;       // flat speculation: some op is not an Add with a one-element path (k_fl_claim<VERIFY>)
  uint32_t pre_done;        // k_pre_ts: workgroups finished (the last lays the ranges out)
  uint32_t fl_nw;           // flat order: words of 64 slots, (range_total + 63) / 64
  uint32_t run_count;       // flat order: ep-runs (scan total)
  uint32_t run_fail;        // flat order: the run tree is deeper than RUN_MAXD (generic list ranking instead)
  uint32_t run_maxd;        // flat order: deepest run
  uint32_t run_lhist[64];   // flat order: runs per depth
  long long rep_inline[2 * REP_INLINE];  // replicas table entries collected by a commit (the first REP_INLINE)
  uint32_t ilr_levels[204];  // host staging: groups, ops and largest private table per level (ilr.hip)
  uint32_t fincr[8];         // incremental flat merge (incr.hip): its flags words, read back with the result
};

#define HIP_CHECK(x)                                                                         \
  do {                                                                                       \
    hipError_t e_ = (x);                                                                     \
    if (e_ != hipSuccess) {                                                                  \
      std::fprintf(stderr, "crdtm HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, \
                   __LINE__);                                                                \
      return CRDTM_E_HIP;                                                                    \
    }                                                                                        \
  } while (0)

inline uint32_t grid_for(uint64_t n, int block = BLOCK, uint32_t cap = 1u << 20) {
  uint64_t g = (n + block - 1) / block;
  if (g == 0) g = 1;
  return static_cast<uint32_t>(g < cap ? g : cap);
}

}  // namespace crdtm
