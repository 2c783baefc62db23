// pdr.hip — per-dict exact replay (PDR) for fresh trees whose dicts see
// Deletes before later Adds, the batches the closed form's guard rejects
// (G_DEL_BEFORE_ADD; configs 1-2 of BASELINE.json).
//
// The reference applies a batch one op at a time (src/CRDTree.elm:224-232,
// :275-295). Ops in different children dicts only interact through path
// resolution: an op's path crosses keys of ancestor dicts, and a key stays
// bound to its original node until that node's first Delete — except when
// findInsertion's copy quirk (src/Internal/Node.elm:93-104)
// later re-fills the tombstoned slot with a copy of a live sibling. So:
//
//  1. K1 (merge.hip, level-synchronous lookup) resolves every path as if no
//     slot were ever re-filled, and tags each op with "reached its leaf dict"
//     or the tombstoned node where the path stopped (Work.tag);
//  2. one lane per children dict replays that dict's reached ops in batch
//     order with the reference's literal addAfter/findInsertion/delete
//     semantics (P2), recording when each key's slot was first re-filled;
//  3. an op whose path stopped at a key re-filled before it ran would have
//     descended into the copy: conflict, and the batch goes to the sequential
//     replay (P3). Otherwise every status is exact;
//  4. assembly (P5): the surviving dicts are the original dicts whose owner
//     chain is live and un-copied, plus one snapshot per copied slot — the
//     deep copy (Replayer::deep_copy) of the source dict as of the copy time,
//     rebuilt by replaying the source dict's op prefix (nested level by
//     level). Slots are numbered by scans and written into TreeDev.
//
// Region layout: original dict D (D = owner op index, n = root) owns the
// slot range [rbase[D], rbase[D+1]) = 1 sentinel + one slot per reached op;
// olist holds the dict's ops in batch order at [rbase[D], rbase[D+1]-1), its
// last position a NONE pad (the sort needs unique keys). Snapshot regions
// follow the originals.

#include "engine.h"

namespace crdtm {

enum : uint8_t { P_TOMB = 1, P_ORPHAN = 2, P_COPY = 4 };

struct PdrRegion {     // per replay slot (originals, then snapshots)
  long long* key;
  uint32_t* next;      // local index in the same region
  uint32_t* src;       // op whose node the slot holds (NONE: sentinel)
  uint32_t* cd;        // children: original dict (owner op) ...
  uint32_t* cb;        // ... as of op index cb (NONE: current)
  uint32_t* ch;        // assembly: snapshot instance of the children
  uint32_t* inst;      // instance owning the slot (NONE: unused room)
  uint8_t* fl;
};

struct PdrInst {       // per instance: originals 0..n (n = root), snapshots n+1+j
  uint32_t* base;
  uint32_t* used;
  uint32_t* src;       // snapshots: source original dict
  uint32_t* bound;     // snapshots: replay the ops < bound
  uint32_t* pi;        // snapshots: parent instance
  uint32_t* pl;        // snapshots: parent local slot
};

struct PdrCtx {
  OpsDev o;
  TsIndex ix;
  const uint32_t* leaf;
  const uint32_t* rbase;  // [n + 2]
  const uint32_t* olist;
  uint32_t* lidx;         // op -> local slot in its original dict
  uint32_t* tcopy;        // node op -> first op whose copy quirk re-filled its key's slot
  PdrRegion R;
  PdrInst I;
};

__device__ __forceinline__ uint32_t pdr_first_op(const PdrCtx& p, uint32_t D) {
  const uint32_t b = p.rbase[D];
  return p.rbase[D + 1] - b > 1 ? p.olist[b] : NONE;
}

// Replay original dict D's ops (ORIG, statuses written) or the op prefix
// < bound of a snapshot, into the region at `base`. Literal semantics of
// Replayer::op's leaf step (merge.hip) on the region.
template <bool ORIG>
__device__ void pdr_replay(const PdrCtx& p, uint8_t* st, uint32_t D, uint32_t bound, uint32_t base, uint32_t inst) {
  const OpsDev& o = p.o;
  const PdrRegion& R = p.R;
  R.key[base] = 0;
  R.next[base] = NONE;
  R.src[base] = NONE;
  R.cd[base] = NONE;
  R.cb[base] = NONE;
  R.ch[base] = NONE;
  R.inst[base] = inst;
  R.fl[base] = P_TOMB;
  uint32_t m = 1;
  const uint32_t ob = p.rbase[D], oe = p.rbase[D + 1] - 1;
  for (uint32_t k = ob; k < oe; ++k) {
    const uint32_t i = p.olist[k];
    if (i >= bound) break;
    uint8_t s;
    if (o.kind[i] == CRDTM_DELETE) {  // deleteHelp
      const uint32_t tg = p.leaf[i];
      if (tg == SENT_T) {
        s = ST_ALREADY;
      } else {
        const uint32_t l = (tg == MISS_T || tg >= i) ? NONE : p.lidx[tg];
        if (l == NONE) {
          s = ST_NOTFOUND;
        } else if (R.fl[base + l] & P_TOMB) {
          s = ST_ALREADY;
        } else {
          R.fl[base + l] |= P_TOMB;
          R.cd[base + l] = NONE;  // Tombstone drops the children
          s = ST_APPLIED;
        }
      }
    } else {  // addAfterHelp: no collision, so the dict holds ts iff an earlier Add of ts reached it
      const long long ts = o.ts[i];
      if (ts == 0 || tsindex_find(p.ix, ts) != i) {
        s = ST_ALREADY;
      } else {
        const uint32_t a = p.leaf[i];
        const uint32_t al = a == SENT_T ? 0u : ((a == MISS_T || a >= i) ? NONE : p.lidx[a]);
        if (al == NONE) {
          s = ST_NOTFOUND;
        } else {
          uint32_t node = al, nk = al;  // findInsertion
          for (;;) {
            const uint32_t rn = R.next[base + node];
            if (rn == NONE) break;
            uint32_t live = rn;
            while (live != NONE && (R.fl[base + live] & P_TOMB)) live = R.next[base + live];
            if (live == NONE) break;
            if (ts > R.key[base + rn]) break;
            nk = rn;
            node = live;
          }
          const uint32_t x = m++;
          const uint32_t gx = base + x;
          R.key[gx] = ts;
          R.next[gx] = R.next[base + node];
          R.src[gx] = i;
          R.cd[gx] = i;
          R.cb[gx] = ORIG ? NONE : bound;
          R.ch[gx] = NONE;
          R.inst[gx] = inst;
          R.fl[gx] = R.fl[base + nk] & P_ORPHAN;
          if (nk == node) {
            R.next[base + node] = x;
          } else {
            // copy quirk: slot nk := copy of node, next = x; the entries after
            // nk up to node drop off the chain when nk was on it
            if (!(R.fl[base + nk] & P_ORPHAN)) {
              for (uint32_t q = R.next[base + nk]; q != NONE; q = R.next[base + q]) {
                R.fl[base + q] |= P_ORPHAN;
                if (q == node) break;
              }
            }
            R.src[base + nk] = R.src[base + node];
            R.fl[base + nk] = (R.fl[base + node] & ~P_ORPHAN) | (R.fl[base + nk] & P_ORPHAN) | P_COPY;
            R.cd[base + nk] = R.cd[base + node];
            R.cb[base + nk] = min(R.cb[base + node], i);
            R.next[base + nk] = x;
            if (ORIG) atomicMin(&p.tcopy[tsindex_find(p.ix, R.key[base + nk])], i);
          }
          if (ORIG) p.lidx[i] = x;
          s = ST_APPLIED;
        }
      }
    }
    if (ORIG) st[i] = s;
  }
  p.I.used[inst] = m;
}

// ---- P1: group the reached ops by leaf dict ----
__global__ void __launch_bounds__(BLOCK) k_pdr_init(uint32_t n, uint32_t* cnt, uint32_t* fill, uint32_t* lidx,
                                                    uint32_t* tcopy) {
  GRID_STRIDE(i, n + 2) {
    cnt[i] = 0;
    fill[i] = 0;
    if (i < n) {
      lidx[i] = NONE;
      tcopy[i] = NONE;
    }
  }
}

__global__ void __launch_bounds__(BLOCK) k_pdr_count(OpsDev o, const uint32_t* tag, const uint32_t* cur,
                                                     uint32_t* cnt) {
  GRID_STRIDE(i, o.n) {
    if (tag[i] == PDR_REACHED) atomicAdd(&cnt[cur[i]], 1u);
  }
}

// region size: sentinel + one slot per reached op; the root dict always exists
__global__ void __launch_bounds__(BLOCK) k_pdr_size(uint32_t n, uint32_t* cnt) {
  GRID_STRIDE(d, n + 1) {
    const uint32_t c = cnt[d];
    cnt[d] = (c || d == n) ? c + 1 : 0u;
  }
}

__global__ void __launch_bounds__(BLOCK) k_pdr_scatter(OpsDev o, const uint32_t* tag, const uint32_t* cur,
                                                       const uint32_t* rbase, uint32_t* fill, uint32_t* olist) {
  GRID_STRIDE(i, o.n) {
    if (tag[i] != PDR_REACHED) continue;
    const uint32_t d = cur[i];
    olist[rbase[d] + atomicAdd(&fill[d], 1u)] = i;  // the pad (NONE) stays last
  }
}

// ---- P2: one lane per original dict ----
__global__ void __launch_bounds__(64) k_pdr_replay_orig(PdrCtx p, uint8_t* st) {
  const uint32_t n = p.o.n;
  const uint32_t D = blockIdx.x * blockDim.x + threadIdx.x;
  if (D > n) return;
  const uint32_t b = p.rbase[D];
  if (p.rbase[D + 1] == b) return;
  p.I.base[D] = b;
  pdr_replay<true>(p, st, D, NONE, b, D);
}

// ---- P3: conflicts ----
__global__ void __launch_bounds__(BLOCK) k_pdr_conflict(uint32_t n, const uint32_t* tag, const uint32_t* tcopy,
                                                        DevResult* dres) {
  GRID_STRIDE(i, n) {
    const uint32_t x = tag[i];
    if (x < n && tcopy[x] < i) atomicOr(&dres->pdr_conflict, 1u);  // rare
  }
}

// batch accounting on the final statuses (k_stats' counters)
__global__ void __launch_bounds__(BLOCK) k_pdr_stats(OpsDev o, const uint8_t* st, long long ts0, DevResult* dres) {
  uint32_t app = 0, alr = 0, err = NONE, own = 0;
  const long long id0 = replica_of(ts0);
  const uint32_t n = o.n;
  const uint32_t stride = gridDim.x * blockDim.x;
  const uint32_t trips = (n + stride - 1) / stride;
  for (uint32_t t = 0; t < trips; ++t) {
    const uint32_t i = t * stride + blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) continue;
    const uint8_t s = st[i];
    if (s == ST_APPLIED) ++app;
    else if (s == ST_ALREADY) ++alr;
    else err = min(err, i);
    if (o.kind[i] == CRDTM_ADD && (s == ST_APPLIED || s == ST_ALREADY) && replica_of(o.ts[i]) == id0) ++own;
  }
  app = block_sum(app);
  alr = block_sum(alr);
  own = block_sum(own);
  err = block_min(err);
  if (threadIdx.x == 0) {
    atomicAdd(&dres->n_applied, app);
    atomicAdd(&dres->n_already, alr);
    atomicAdd(&dres->own_ok_adds, own);
    if (err != NONE) atomicMin(&dres->err_index, err);
  }
}

__global__ void k_pdr_stats_reset(DevResult* d) {
  d->n_applied = 0;
  d->n_already = 0;
  d->own_ok_adds = 0;
  d->err_index = NONE;
  d->pdr_jobs = 0;
  d->pdr_overflow = 0;
}

// ---- P5: assembly ----
// alive[D]: original dict D is reachable in the final state (its owner is a
// live, un-copied node of an alive dict). ok/up pointer jumping as in
// k_dict_alive_*.
__global__ void __launch_bounds__(BLOCK) k_pdr_alive_init(PdrCtx p, const uint32_t* addpar, uint8_t* ok,
                                                          uint32_t* up) {
  const uint32_t n = p.o.n;
  GRID_STRIDE(d, n + 1) {
    if (d == n) {
      ok[d] = 1;
      up[d] = n;
      continue;
    }
    uint8_t v = 0;
    uint32_t P = n;
    if (p.rbase[d + 1] != p.rbase[d]) {
      P = addpar[d];
      const uint32_t l = p.lidx[d];
      v = (l != NONE && !(p.R.fl[p.rbase[P] + l] & (P_TOMB | P_COPY))) ? 1 : 0;
    }
    ok[d] = v;
    up[d] = P;
  }
}

__global__ void __launch_bounds__(BLOCK) k_pdr_alive_jump(uint32_t n, uint8_t* ok, uint32_t* up) {
  GRID_STRIDE(d, n + 1) {
    const uint32_t u = up[d];
    if (!ok[u]) ok[d] = 0;
    up[d] = up[u];
  }
}

// A live slot whose children are a frozen (dict, bound) view gets a snapshot
// job when that view is non-empty. Slots [s0, s1) of the last replayed regions.
__global__ void __launch_bounds__(BLOCK) k_pdr_jobs(PdrCtx p, const uint8_t* ok, uint32_t s0, uint32_t s1,
                                                    uint32_t jcap, uint32_t scap_left, DevResult* dres) {
  const uint32_t n = p.o.n;
  GRID_STRIDE(k, s1 - s0) {
    const uint32_t g = s0 + k;
    const uint32_t I = p.R.inst[g];
    if (I == NONE) continue;
    if (I <= n && !ok[I]) continue;  // a dead original dict
    const uint8_t f = p.R.fl[g];
    if (f & P_TOMB) continue;        // (sentinels too)
    if (I <= n && !(f & P_COPY)) continue;  // children = the live original dict
    const uint32_t cd = p.R.cd[g], cb = p.R.cb[g];
    const uint32_t f0 = pdr_first_op(p, cd);
    if (f0 == NONE || f0 >= cb) continue;  // the copy is an empty dict (implicit)
    const uint32_t j = atomicAdd(&dres->pdr_jobs, 1u);
    if (j >= jcap) {
      atomicOr(&dres->pdr_overflow, 1u);
      continue;
    }
    const uint32_t J = n + 1 + j;
    p.I.src[J] = cd;
    p.I.bound[J] = cb;
    p.I.pi[J] = I;
    p.I.pl[J] = g - p.I.base[I];
    p.R.ch[g] = J;
  }
  (void)scap_left;
}

__global__ void __launch_bounds__(BLOCK) k_pdr_job_size(PdrCtx p, uint32_t j0, uint32_t j1, uint32_t* sz) {
  const uint32_t n = p.o.n;
  GRID_STRIDE(k, j1 - j0 + 1) {
    if (k == j1 - j0) {
      sz[k] = 0;
      continue;
    }
    const uint32_t d = p.I.src[n + 1 + j0 + k];
    sz[k] = p.rbase[d + 1] - p.rbase[d];
  }
}

__global__ void __launch_bounds__(64) k_pdr_replay_snap(PdrCtx p, uint32_t j0, uint32_t j1, const uint32_t* off,
                                                        uint32_t s0) {
  const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= j1 - j0) return;
  const uint32_t J = p.o.n + 1 + j0 + k;
  const uint32_t b = s0 + off[k];
  p.I.base[J] = b;
  pdr_replay<false>(p, nullptr, p.I.src[J], p.I.bound[J], b, J);
}

// instance order: root first, then originals 0..n-1, then snapshots
__device__ __forceinline__ uint32_t pdr_pos(uint32_t I, uint32_t n) { return I == n ? 0u : (I < n ? I + 1 : I); }

__global__ void __launch_bounds__(BLOCK) k_pdr_inst_flags(PdrCtx p, const uint8_t* ok, uint32_t njobs,
                                                          uint32_t* dflag, uint32_t* dsize) {
  const uint32_t n = p.o.n;
  GRID_STRIDE(I, n + 1 + njobs + 1) {
    if (I == n + 1 + njobs) {  // scan tail
      dflag[I] = 0;
      dsize[I] = 0;
      continue;
    }
    const bool inst = I > n || (ok[I] && p.rbase[I + 1] != p.rbase[I]);
    const uint32_t q = pdr_pos(I, n);
    dflag[q] = inst ? 1u : 0u;
    dsize[q] = inst ? p.I.used[I] : 0u;
  }
}

__global__ void __launch_bounds__(BLOCK) k_pdr_write(PdrCtx p, const uint8_t* ok, const uint32_t* addpar,
                                                     const uint32_t* did, const uint32_t* sbase,
                                                     const uint32_t* logidx, uint32_t S, TreeDev T) {
  const uint32_t n = p.o.n;
  GRID_STRIDE(g, S) {
    const uint32_t I = p.R.inst[g];
    if (I == NONE) continue;
    if (I <= n && !(ok[I])) continue;
    const uint32_t q = pdr_pos(I, n);
    const uint32_t l = g - p.I.base[I];
    const uint32_t sb = sbase[q];
    const uint32_t d = did[q];
    const uint32_t s = sb + l;
    const uint8_t f = p.R.fl[g];
    const uint32_t nx = p.R.next[g];
    T.s_key[s] = p.R.key[g];
    T.s_dict[s] = d;
    T.s_next[s] = nx == NONE ? NONE : sb + nx;
    uint32_t child = NONE;
    if (l == 0) {
      T.s_src[s] = NONE;
      T.s_flags[s] = F_TOMB | F_SENT;
      T.d_sent[d] = s;
      uint32_t owner = NONE;
      if (I > n) {
        owner = sbase[pdr_pos(p.I.pi[I], n)] + p.I.pl[I];
      } else if (I < n) {
        owner = sbase[pdr_pos(addpar[I], n)] + p.lidx[I];
      }
      T.d_owner[d] = owner;
    } else {
      T.s_src[s] = logidx[p.R.src[g]];
      T.s_flags[s] = ((f & P_TOMB) ? F_TOMB : 0) | ((f & P_ORPHAN) ? F_ORPHAN : 0);
      if (!(f & P_TOMB)) {
        if (I > n || (f & P_COPY)) {
          const uint32_t J = p.R.ch[g];
          if (J != NONE) child = did[pdr_pos(J, n)];
        } else {
          const uint32_t y = p.R.src[g];  // a live original node: its own dict
          if (p.rbase[y + 1] != p.rbase[y]) child = did[pdr_pos(y, n)];
        }
      }
    }
    T.s_child[s] = child;
  }
}

__global__ void __launch_bounds__(BLOCK) k_pdr_logidx(OpsDev o, const uint8_t* st, uint32_t* a) {
  GRID_STRIDE(i, o.n) a[i] = st[i] == ST_APPLIED ? 1u : 0u;
}

// Host driver. *handled = false: conflict or no room, the caller replays
// the batch sequentially (statuses in `st` are then scratch).
int pdr_apply(crdtm_tree* t, const OpsDev& o, const PdrIn& in, uint8_t* st, crdtm_result* res, bool* handled) {
  crdtm_ctx* c = t->ctx;
  hipStream_t s = c->stream;
  Arena& ws = c->ws;
  DevResult* dr = c->dres;
  const uint32_t n = o.n;
  const uint32_t g = grid_for(n);
  *handled = false;
  const size_t arena_mark = ws.used;
  int r;

  PdrCtx p;
  p.o = o;
  p.ix = in.ix;
  p.leaf = in.leaf;
  uint32_t* rbase = ws.alloc<uint32_t>(n + 2);
  uint32_t* fill = ws.alloc<uint32_t>(n + 2);
  p.lidx = ws.alloc<uint32_t>(n);
  p.tcopy = ws.alloc<uint32_t>(n);
  LAUNCH(k_pdr_init, dim3(grid_for(n + 2)), dim3(BLOCK), 0, s, n, rbase, fill, p.lidx, p.tcopy);
  LAUNCH(k_pdr_count, dim3(g), dim3(BLOCK), 0, s, o, in.tag, in.cur, rbase);
  LAUNCH(k_pdr_size, dim3(grid_for(n + 1)), dim3(BLOCK), 0, s, n, rbase);
  uint32_t* rtot = &dr->pdr_slots;
  if ((r = scan_excl_u32(rbase, rbase, n + 2, rtot, ws, s))) return r;
  if ((r = sync_read(c))) return r;
  const uint32_t R0 = c->hres->pdr_slots;  // original regions
  p.rbase = rbase;
  uint32_t* olist = ws.alloc<uint32_t>(R0);
  p.olist = olist;
  HIP_CHECK(hipMemsetAsync(olist, 0xFF, static_cast<size_t>(R0) * sizeof(uint32_t), s));
  LAUNCH(k_pdr_scatter, dim3(grid_for(n)), dim3(BLOCK), 0, s, o, in.tag, in.cur, rbase, fill, olist);
  if ((r = segmented_sort_asc_id(rbase, n + 1, olist, R0, ws, s, dr))) return r;

  // slot room: originals + snapshots (bounded; overflow -> sequential replay)
  const uint64_t scap64 = std::min<uint64_t>(2ULL * R0 + 4096, 0xF0000000ULL);
  const uint32_t SCAP = static_cast<uint32_t>(scap64);
  const uint32_t JCAP = std::max<uint32_t>(1024u, n);
  PdrRegion& R = p.R;
  R.key = ws.alloc<long long>(SCAP);
  R.next = ws.alloc<uint32_t>(SCAP);
  R.src = ws.alloc<uint32_t>(SCAP);
  R.cd = ws.alloc<uint32_t>(SCAP);
  R.cb = ws.alloc<uint32_t>(SCAP);
  R.ch = ws.alloc<uint32_t>(SCAP);
  R.inst = ws.alloc<uint32_t>(SCAP);
  R.fl = ws.alloc<uint8_t>(SCAP);
  const uint64_t ICAP = static_cast<uint64_t>(n) + 1 + JCAP;
  PdrInst& I = p.I;
  I.base = ws.alloc<uint32_t>(ICAP);
  I.used = ws.alloc<uint32_t>(ICAP);
  I.src = ws.alloc<uint32_t>(ICAP);
  I.bound = ws.alloc<uint32_t>(ICAP);
  I.pi = ws.alloc<uint32_t>(ICAP);
  I.pl = ws.alloc<uint32_t>(ICAP);
  HIP_CHECK(hipMemsetAsync(R.inst, 0xFF, static_cast<size_t>(SCAP) * sizeof(uint32_t), s));

  // ---- P2 + P3 ----
  LAUNCH(k_pdr_replay_orig, dim3((n + 1 + 63) / 64), dim3(64), 0, s, p, st);
  LAUNCH(k_pdr_stats_reset, dim3(1), dim3(1), 0, s, dr);
  HIP_CHECK(hipMemsetAsync(&dr->pdr_conflict, 0, sizeof(uint32_t), s));
  LAUNCH(k_pdr_conflict, dim3(grid_for(n, BLOCK, 2048)), dim3(BLOCK), 0, s, n, in.tag, p.tcopy, dr);
  LAUNCH(k_pdr_stats, dim3(grid_for(n, BLOCK, 2048)), dim3(BLOCK), 0, s, o, st, t->timestamp, dr);
  if ((r = sync_read(c))) return r;
  const DevResult h1 = *c->hres;
  if (h1.pdr_conflict) {
    ws.used = arena_mark;
    return CRDTM_OK;
  }
  const long long new_ts = t->timestamp + h1.own_ok_adds;
  if (replica_of(new_ts) != replica_of(t->timestamp)) {
    ws.used = arena_mark;
    return CRDTM_OK;
  }
  *handled = true;
  res->path_taken = CRDTM_PATH_DICT_REPLAY;
  if (h1.err_index != NONE) {
    uint8_t est = 0;
    HIP_CHECK(hipMemcpy(&est, st + h1.err_index, 1, hipMemcpyDeviceToHost));
    res->code = est == ST_INVALID ? CRDTM_INVALID_PATH : CRDTM_OPERATION_FAILED;
    res->err_index = h1.err_index;
    return CRDTM_OK;
  }
  res->n_applied = h1.n_applied;
  res->n_already = h1.n_already;

  // ---- P5: alive originals, snapshot jobs level by level ----
  uint8_t* ok = ws.alloc<uint8_t>(n + 1);
  uint32_t* up = ws.alloc<uint32_t>(n + 1);
  LAUNCH(k_pdr_alive_init, dim3(grid_for(n + 1)), dim3(BLOCK), 0, s, p, in.addpar, ok, up);
  for (uint32_t span = 1; span < in.maxlen + 1; span <<= 1)
    LAUNCH(k_pdr_alive_jump, dim3(grid_for(n + 1)), dim3(BLOCK), 0, s, n, ok, up);
  uint32_t s0 = 0, s1 = R0, j0 = 0;
  uint32_t* joff = ws.alloc<uint32_t>(JCAP + 1);
  for (uint32_t level = 0;; ++level) {
    LAUNCH(k_pdr_jobs, dim3(grid_for(s1 - s0)), dim3(BLOCK), 0, s, p, ok, s0, s1, JCAP, SCAP - s1, dr);
    if ((r = sync_read(c))) return r;
    if (c->hres->pdr_overflow || level > in.maxlen + 1) {  // no room: sequential replay
      *handled = false;
      ws.used = arena_mark;
      return CRDTM_OK;
    }
    const uint32_t j1 = c->hres->pdr_jobs;
    if (j1 == j0) break;
    LAUNCH(k_pdr_job_size, dim3(grid_for(j1 - j0 + 1)), dim3(BLOCK), 0, s, p, j0, j1, joff);
    if ((r = scan_excl_u32(joff, joff, j1 - j0 + 1, &dr->pdr_slots, ws, s))) return r;
    if ((r = sync_read(c))) return r;
    const uint64_t need = static_cast<uint64_t>(s1) + c->hres->pdr_slots;
    if (need > SCAP) {
      *handled = false;
      ws.used = arena_mark;
      return CRDTM_OK;
    }
    LAUNCH(k_pdr_replay_snap, dim3((j1 - j0 + 63) / 64), dim3(64), 0, s, p, j0, j1, joff, s1);
    s0 = s1;
    s1 = static_cast<uint32_t>(need);
    j0 = j1;
  }
  const uint32_t nj = j0;

  // ---- numbering ----
  const uint32_t NI = n + 1 + nj;
  uint32_t* did = ws.alloc<uint32_t>(NI + 1);
  uint32_t* sbase = ws.alloc<uint32_t>(NI + 1);
  LAUNCH(k_pdr_inst_flags, dim3(grid_for(NI + 1)), dim3(BLOCK), 0, s, p, ok, nj, did, sbase);
  if ((r = scan_excl_u32(did, did, NI + 1, &dr->pdr_dicts, ws, s))) return r;
  if ((r = scan_excl_u32(sbase, sbase, NI + 1, &dr->pdr_slots, ws, s))) return r;
  uint32_t* logidx = ws.alloc<uint32_t>(n + 1);
  LAUNCH(k_pdr_logidx, dim3(g), dim3(BLOCK), 0, s, o, st, logidx);
  if ((r = scan_excl_u32(logidx, logidx, n, nullptr, ws, s))) return r;
  if ((r = sync_read(c))) return r;
  const uint32_t n_dicts = c->hres->pdr_dicts, n_slots = c->hres->pdr_slots;
  TreeCaps need = t->cap;
  need.slots = std::max<uint64_t>(need.slots, n_slots + 1ULL);
  need.dicts = std::max<uint64_t>(need.dicts, n_dicts + 1ULL);
  need.log = std::max<uint64_t>(need.log, t->log_n + h1.n_applied + 1);
  need.lpath = std::max<uint64_t>(need.lpath, t->log_npath + o.n_path + 1);
  if (need.slots > t->cap.slots || need.dicts > t->cap.dicts || need.log > t->cap.log || need.lpath > t->cap.lpath) {
    if ((r = grow_tree(t, need))) return r;
  }
  LAUNCH(k_pdr_write, dim3(grid_for(s1)), dim3(BLOCK), 0, s, p, ok, in.addpar, did, sbase, logidx, s1, t->d);
  if ((r = post_pass(t, o, st, ws))) return r;
  t->n_slots = n_slots;
  t->n_dicts = n_dicts;
  t->timestamp = new_ts;
  t->doc_valid = false;
  res->code = CRDTM_OK;
  return CRDTM_OK;
}

}  // namespace crdtm
