// synth.cpp — deterministic synthetic CRDTree op streams.
//
// Models the reference's local editing API as used by replicas
// (src/CRDTree.elm:142-216): a replica "types" after its own last node
// (add, :151-153), sometimes anchors after a node it can see (addAfter,
// :166-168), sometimes opens a branch (addBranch, :180-186), and deletes
// visible nodes (delete, :199-216). Timestamps follow the reference's scheme
// ts = replicaId * 2^32 + counter (src/CRDTree.elm:137, :348-350). Views lag
// by a window of W generated ops, so inserts are genuinely concurrent. The
// batch order is the causal generation order: every op only references nodes
// generated before it, so a reference `apply (Batch ops)` never fails.

#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <algorithm>
#include <new>
#include <thread>
#include <vector>

#include "../../include/crdtm.h"

namespace {

struct Rng {  // splitmix64: deterministic, identical on every host
  uint64_t s;
  explicit Rng(uint64_t seed) : s(seed) {}
  uint64_t next() {
    uint64_t z = (s += 0x9E3779B97F4A7C15ULL);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
  }
  uint64_t below(uint64_t n) { return n ? next() % n : 0; }
  double uniform() { return (next() >> 11) * (1.0 / 9007199254740992.0); }
};

struct GNode {
  int64_t key;
  int32_t parent;  // node index, -1 = root
  uint32_t gen_step;
  uint32_t del_step;  // UINT32_MAX = live
  uint16_t depth;     // root children = 1
  uint16_t nchild;
};

struct Out {
  std::vector<uint8_t> kind;
  std::vector<int64_t> ts;
  std::vector<uint32_t> off{0};
  std::vector<int64_t> path;
  std::vector<uint32_t> val;
  std::vector<uint32_t> tree;
};

void pathOf(const std::vector<GNode>& nodes, int32_t n, std::vector<int64_t>& tmp) {
  tmp.clear();
  while (n >= 0) { tmp.push_back(nodes[n].key); n = nodes[n].parent; }
  // reverse in place: root-first
  for (size_t i = 0, j = tmp.size(); i + 1 < j; ++i, --j) std::swap(tmp[i], tmp[j - 1]);
}

void emitAdd(Out& o, int64_t ts, const std::vector<GNode>& nodes, int32_t parent, int64_t anchor, uint32_t val,
             uint32_t doc, std::vector<int64_t>& tmp) {
  pathOf(nodes, parent, tmp);
  o.kind.push_back(CRDTM_ADD);
  o.ts.push_back(ts);
  for (int64_t k : tmp) o.path.push_back(k);
  o.path.push_back(anchor);
  o.off.push_back(static_cast<uint32_t>(o.path.size()));
  o.val.push_back(val);
  o.tree.push_back(doc);
}

void emitDel(Out& o, const std::vector<GNode>& nodes, int32_t n, uint32_t doc, std::vector<int64_t>& tmp) {
  pathOf(nodes, n, tmp);
  o.kind.push_back(CRDTM_DELETE);
  o.ts.push_back(0);
  for (int64_t k : tmp) o.path.push_back(k);
  o.off.push_back(static_cast<uint32_t>(o.path.size()));
  o.val.push_back(0);
  o.tree.push_back(doc);
}

// Typing model (configs 1, 2, 3, 5).
void genTyping(const crdtm_synth_params& p, uint64_t seed, uint32_t doc, Out& o) {
  Rng rng(seed);
  const uint32_t R = p.replicas ? p.replicas : 1;
  const uint64_t W = p.window;
  std::vector<GNode> nodes;
  nodes.reserve(p.n_ops);
  std::vector<uint32_t> counter(R + 1, 1);
  std::vector<int32_t> ownLast(R + 1, -1), curParent(R + 1, -1);
  std::vector<int64_t> tmp;
  size_t known = 0;  // nodes[0..known) are visible to every replica
  const uint64_t nDel = static_cast<uint64_t>(p.n_ops * p.p_delete);
  const uint64_t nAdd = p.n_ops - (p.deletes_last ? nDel : 0);
  uint64_t emitted = 0;
  auto visible = [&](uint64_t s, const GNode& g) { return g.del_step == UINT32_MAX || g.del_step + W > s; };
  for (uint64_t s = 0; emitted < nAdd; ++s) {
    while (known < nodes.size() && nodes[known].gen_step + W <= s) ++known;
    const uint32_t r = 1 + static_cast<uint32_t>(rng.below(R));
    if (!p.deletes_last && p.p_delete > 0 && known > 0 && rng.uniform() < p.p_delete) {
      int32_t pick = -1;
      for (int tries = 0; tries < 8 && pick < 0; ++tries) {
        uint64_t c = rng.below(known);
        const GNode& g = nodes[c];
        if (visible(s, g) && g.nchild == 0) pick = static_cast<int32_t>(c);
      }
      if (pick >= 0) {
        emitDel(o, nodes, pick, doc, tmp);
        if (nodes[pick].del_step == UINT32_MAX) nodes[pick].del_step = static_cast<uint32_t>(s);
        ++emitted;
        continue;
      }
    }
    int32_t parent, anchorNode;
    if (ownLast[r] >= 0 && rng.uniform() < p.p_continue) {
      parent = curParent[r];
      anchorNode = ownLast[r];
    } else if (curParent[r] >= 0 && ownLast[r] < 0) {
      parent = curParent[r];  // first char of a freshly opened branch
      anchorNode = -1;
    } else if (known > 0) {
      anchorNode = -1;
      for (int tries = 0; tries < 8 && anchorNode < 0; ++tries) {
        uint64_t c = rng.below(known);
        if (visible(s, nodes[c])) anchorNode = static_cast<int32_t>(c);
      }
      parent = anchorNode >= 0 ? nodes[anchorNode].parent : -1;
    } else {
      parent = -1;
      anchorNode = -1;
    }
    const int64_t ts = (static_cast<int64_t>(r) << 32) | counter[r]++;
    const int64_t anchor = anchorNode >= 0 ? nodes[anchorNode].key : 0;
    emitAdd(o, ts, nodes, parent, anchor, static_cast<uint32_t>('a' + (s % 26)), doc, tmp);
    GNode g;
    g.key = ts;
    g.parent = parent;
    g.gen_step = static_cast<uint32_t>(s);
    g.del_step = UINT32_MAX;
    g.depth = static_cast<uint16_t>(parent >= 0 ? nodes[parent].depth + 1 : 1);
    g.nchild = 0;
    if (parent >= 0 && nodes[parent].nchild < UINT16_MAX) nodes[parent].nchild++;
    nodes.push_back(g);
    const int32_t x = static_cast<int32_t>(nodes.size() - 1);
    ownLast[r] = x;
    curParent[r] = parent;
    if (p.max_depth > 1 && g.depth + 1u <= p.max_depth && rng.uniform() < p.p_branch) {
      curParent[r] = x;  // addBranch: cursor := path ++ [0]
      ownLast[r] = -1;
    }
    ++emitted;
  }
  if (p.deletes_last) {
    // Deletes of distinct random nodes, after every Add (partial Fisher-Yates).
    std::vector<uint32_t> idx(nodes.size());
    for (size_t i = 0; i < idx.size(); ++i) idx[i] = static_cast<uint32_t>(i);
    for (uint64_t k = 0; k < nDel && k < idx.size(); ++k) {
      uint64_t j = k + rng.below(idx.size() - k);
      std::swap(idx[k], idx[j]);
      emitDel(o, nodes, static_cast<int32_t>(idx[k]), doc, tmp);
    }
  }
}

// Deep-tree model (config 4): parent uniform among nodes with depth < max_depth
// and < max_children children; anchor = a random existing child or the head.
void genDeep(const crdtm_synth_params& p, uint64_t seed, uint32_t doc, Out& o) {
  Rng rng(seed);
  const uint32_t R = p.replicas ? p.replicas : 16;
  const uint32_t C = p.max_children;
  const uint64_t nDel = static_cast<uint64_t>(p.n_ops * p.p_delete);
  const uint64_t nAdd = p.n_ops - nDel;
  std::vector<GNode> nodes;
  nodes.reserve(nAdd);
  std::vector<int32_t> kids;  // [node+1][C] (slot 0 = root)
  kids.assign((nAdd + 1) * C, -1);
  std::vector<uint16_t> rootKidsN(1, 0);
  std::vector<int32_t> eligible;  // node index + 1 (0 = root)
  eligible.reserve(nAdd + 1);
  eligible.push_back(0);
  std::vector<uint32_t> eligPos(nAdd + 1, 0);
  std::vector<uint32_t> counter(R + 1, 1);
  std::vector<int64_t> tmp;
  auto nchild = [&](int32_t pn) -> uint16_t { return pn == 0 ? rootKidsN[0] : nodes[pn - 1].nchild; };
  // Interleaved variant (deletes_last = 0, SURVEY.md 8d config 4's second
  // stream): each step is a Delete with probability (deletes left) / (ops
  // left), so the batch holds exactly nAdd Adds and nDel Deletes, spread
  // uniformly. A Delete targets a uniformly chosen live leaf (like a replica
  // deleting a visible node without children, the typing model's rule), which
  // then stops being a parent candidate: every op of the stream applies, and
  // later Adds keep landing in dicts that already hold tombstones — with
  // anchors that may be those deleted siblings (findInsertion's tombstone skip
  // and copy quirk, src/Internal/Node.elm:93-104).
  const bool inter = !p.deletes_last && nDel > 0;
  std::vector<int32_t> leaves;    // live nodes without children
  std::vector<uint32_t> leafPos;  // node -> position in `leaves`, UINT32_MAX = not a leaf
  std::vector<uint8_t> inElig;    // node + 1 -> listed in `eligible`
  if (inter) {
    leaves.reserve(nAdd);
    leafPos.assign(nAdd, UINT32_MAX);
    inElig.assign(nAdd + 1, 0);
    inElig[0] = 1;
  }
  auto dropLeaf = [&](int32_t v) {
    const uint32_t pos = leafPos[v];
    leaves[pos] = leaves.back();
    leafPos[leaves[pos]] = pos;
    leaves.pop_back();
    leafPos[v] = UINT32_MAX;
  };
  uint64_t delLeft = inter ? nDel : 0;
  for (uint64_t s = 0, addsDone = 0; addsDone < nAdd || (delLeft > 0 && !leaves.empty()); ++s) {
    if (inter && delLeft > 0 && !leaves.empty() &&
        (addsDone == nAdd || rng.below(delLeft + (nAdd - addsDone)) < delLeft)) {
      const int32_t v = leaves[rng.below(leaves.size())];
      emitDel(o, nodes, v, doc, tmp);
      dropLeaf(v);
      const int32_t x = v + 1;
      if (inElig[x]) {  // no longer a parent candidate
        const uint32_t pos = eligPos[x];
        eligible[pos] = eligible.back();
        eligPos[eligible[pos]] = pos;
        eligible.pop_back();
        inElig[x] = 0;
      }
      --delLeft;
      continue;
    }
    ++addsDone;
    if (eligible.empty()) break;
    const uint64_t ei = rng.below(eligible.size());
    const int32_t pn = eligible[ei];  // parent node + 1
    const uint16_t k = nchild(pn);
    const uint64_t a = rng.below(k + 1u);
    const int64_t anchor = a == 0 ? 0 : nodes[kids[static_cast<size_t>(pn) * C + (a - 1)]].key;
    const uint32_t r = 1 + static_cast<uint32_t>(rng.below(R));
    const int64_t ts = (static_cast<int64_t>(r) << 32) | counter[r]++;
    emitAdd(o, ts, nodes, pn - 1, anchor, static_cast<uint32_t>(s & 0xffffff), doc, tmp);
    GNode g;
    g.key = ts;
    g.parent = pn - 1;
    g.gen_step = static_cast<uint32_t>(s);
    g.del_step = UINT32_MAX;
    g.depth = static_cast<uint16_t>(pn == 0 ? 1 : nodes[pn - 1].depth + 1);
    g.nchild = 0;
    nodes.push_back(g);
    const int32_t x = static_cast<int32_t>(nodes.size());  // +1 encoded
    kids[static_cast<size_t>(pn) * C + k] = x - 1;
    if (pn == 0) rootKidsN[0]++; else nodes[pn - 1].nchild++;
    if (nchild(pn) >= C) {  // parent full: swap-remove from eligible
      const uint32_t pos = static_cast<uint32_t>(ei);
      eligible[pos] = eligible.back();
      eligPos[eligible[pos]] = pos;
      eligible.pop_back();
      if (inter) inElig[pn] = 0;
    }
    if (g.depth < p.max_depth) {
      eligPos[x] = static_cast<uint32_t>(eligible.size());
      eligible.push_back(x);
      if (inter) inElig[x] = 1;
    }
    if (inter) {
      if (pn > 0 && leafPos[pn - 1] != UINT32_MAX) dropLeaf(pn - 1);
      leafPos[x - 1] = static_cast<uint32_t>(leaves.size());
      leaves.push_back(x - 1);
    }
  }
  if (inter) return;
  std::vector<uint32_t> idx(nodes.size());
  for (size_t i = 0; i < idx.size(); ++i) idx[i] = static_cast<uint32_t>(i);
  for (uint64_t k = 0; k < nDel && k < idx.size(); ++k) {
    uint64_t j = k + rng.below(idx.size() - k);
    std::swap(idx[k], idx[j]);
    emitDel(o, nodes, static_cast<int32_t>(idx[k]), doc, tmp);
  }
}

template <class T>
T* dup(const std::vector<T>& v) {
  T* p = static_cast<T*>(std::malloc(v.size() * sizeof(T) + 8));
  if (p && !v.empty()) std::memcpy(p, v.data(), v.size() * sizeof(T));
  return p;
}

}  // namespace

extern "C" int crdtm_synth(const crdtm_synth_params* p, crdtm_ops** out) {
  if (!p || !out || p->n_ops == 0) return CRDTM_E_ARG;
  try {
    Out o;
    const uint64_t docs = p->n_docs ? p->n_docs : 1;
    auto gen = [p, docs](uint64_t d0, uint64_t d1, Out& out) {
      out.kind.reserve(p->n_ops * (d1 - d0));
      out.ts.reserve(p->n_ops * (d1 - d0));
      out.val.reserve(p->n_ops * (d1 - d0));
      out.off.reserve(p->n_ops * (d1 - d0) + 1);
      out.tree.reserve(p->n_ops * (d1 - d0));
      for (uint64_t d = d0; d < d1; ++d) {
        const uint64_t id = p->doc_base + d;
        const uint64_t seed = p->seed ^ (0xD1B54A32D192ED03ULL * (id + 1));
        const bool single = docs == 1 && p->doc_base == 0;
        if (p->max_children > 0) genDeep(*p, single ? p->seed : seed, static_cast<uint32_t>(id), out);
        else genTyping(*p, single ? p->seed : seed, static_cast<uint32_t>(id), out);
      }
    };
    // documents are independent streams (their own seeds): many documents are
    // generated on up to 16 threads and concatenated in document order
    const uint64_t nt = std::min<uint64_t>({16, std::max(1u, std::thread::hardware_concurrency()),
                                             docs * p->n_ops >= (1u << 20) ? docs : 1});
    if (nt <= 1) {
      gen(0, docs, o);
    } else {
      std::vector<Out> part(nt);
      std::vector<std::thread> th;
      std::vector<int> failed(nt, 0);
      for (uint64_t t = 0; t < nt; ++t)
        th.emplace_back([&, t] {
          try {
            gen(docs * t / nt, docs * (t + 1) / nt, part[t]);
          } catch (const std::bad_alloc&) {
            failed[t] = 1;
          }
        });
      for (auto& x : th) x.join();
      for (int f : failed)
        if (f) throw std::bad_alloc();
      for (auto& q : part) {
        const uint32_t base = static_cast<uint32_t>(o.path.size());
        o.kind.insert(o.kind.end(), q.kind.begin(), q.kind.end());
        o.ts.insert(o.ts.end(), q.ts.begin(), q.ts.end());
        o.val.insert(o.val.end(), q.val.begin(), q.val.end());
        o.tree.insert(o.tree.end(), q.tree.begin(), q.tree.end());
        o.path.insert(o.path.end(), q.path.begin(), q.path.end());
        for (size_t i = 1; i < q.off.size(); ++i) o.off.push_back(base + q.off[i]);
        Out().kind.swap(q.kind);
        q = Out();
      }
    }
    auto* r = static_cast<crdtm_ops*>(std::calloc(1, sizeof(crdtm_ops)));
    if (!r) return CRDTM_E_NOMEM;
    r->n_ops = o.kind.size();
    r->n_path = o.path.size();
    r->kind = dup(o.kind);
    r->ts = dup(o.ts);
    r->path_off = dup(o.off);
    r->path = dup(o.path);
    r->val = dup(o.val);
    r->tree = (docs > 1 || p->doc_base > 0) ? dup(o.tree) : nullptr;
    *out = r;
    return CRDTM_OK;
  } catch (const std::bad_alloc&) {
    return CRDTM_E_NOMEM;
  }
}

extern "C" int crdtm_ops_free(crdtm_ops* ops) {
  if (!ops) return CRDTM_OK;
  std::free(ops->kind);
  std::free(ops->ts);
  std::free(ops->path_off);
  std::free(ops->path);
  std::free(ops->val);
  std::free(ops->tree);
  std::free(ops);
  return CRDTM_OK;
}
