// oracle/crdtree_oracle.cpp
//
// TEST INFRASTRUCTURE ONLY — the CPU restatement of the Elm reference
// (maca/crdt-replicated-tree 5.0.0) used as the parity checker. Only tests/,
// __graft_entry__.smoke() and bench.py's cpu_baseline leg may load this
// library. The product path (crdt-graph_amd/) never links or calls it.
//
// The reference cannot be compiled here (Elm 0.19, no compiler, no package
// cache), so this is a line-by-line restatement over mutable
// maps. Every function cites the Elm source it follows. Elm values are
// persistent; a mutable restatement is equivalent as long as (1) every error
// is detected before the first mutation of an op (true for addAfterHelp,
// deleteHelp and update), (2) a top-level `apply` that fails leaves the tree
// untouched (we apply to a deep copy and swap on success), and (3) the one
// place Elm shares a node value between two dict slots — the findInsertion
// "copy quirk" — makes a deep copy.
//
// Pinned by: the 83 reference tests transcribed in tests/test_oracle_kat.py
// and the hand-traced vectors of SURVEY.md Appendix C.

#include <algorithm>
#include <cstdint>
#include <cstring>
#include <map>
#include <memory>
#include <utility>
#include <vector>

namespace {

enum Kind : int { ROOT = 0, NODE = 1, TOMB = 2 };
// Internal.Node.Error (src/Internal/Node.elm:35-38) + Ok
enum NErr : int { N_OK = 0, N_NOTFOUND = 1, N_ALREADY = 2, N_INVALID = 3 };
// CRDTree.Error (src/CRDTree.elm:104-107) + Ok
enum TErr : int { T_OK = 0, T_INVALID_PATH = 1, T_NOT_FOUND = 2, T_OPERATION_FAILED = 3 };

struct Node;
// Children a = Dict Int (Node a)   (src/Internal/Node.elm:25-26). std::map keeps
// Elm Dict's ascending key order for the canonical dump.
using Dict = std::map<int64_t, Node>;

// type Node a = Root (Children a) | Node a (Children a) (Array Int) (Maybe Int)
//             | Tombstone (Array Int) (Maybe Int)        (src/Internal/Node.elm:29-32)
struct Node {
  int kind = ROOT;
  uint32_t val = 0;             // value handle (Node only)
  std::vector<int64_t> path;    // Node/Tombstone
  bool has_next = false;        // Maybe Int
  int64_t next = 0;
  Dict children;                // Root/Node (Tombstone: always empty)
};

// emptyChildren = Dict.singleton 0 (Tombstone Array.empty Nothing)  (src/Internal/Node.elm:46-48)
Dict emptyChildren() {
  Dict d;
  Node s;
  s.kind = TOMB;
  d.emplace(0, std::move(s));
  return d;
}

// children (src/Internal/Node.elm:231-241): Tombstone -> Dict.empty
// child ts node = children node |> Dict.get ts   (src/Internal/Node.elm:284-286)
Node* child(int64_t ts, Node& n) {
  if (n.kind == TOMB) return nullptr;
  auto it = n.children.find(ts);
  return it == n.children.end() ? nullptr : &it->second;
}

// nextNode (src/Internal/Node.elm:257-268): follow `next` keys, skipping Tombstones.
Node* nextNode(Node* node, Dict& c) {
  for (;;) {
    if (node->kind == ROOT || !node->has_next) return nullptr;  // next (Root _) = Nothing
    auto it = c.find(node->next);
    if (it == c.end()) return nullptr;
    if (it->second.kind == TOMB) { node = &it->second; continue; }
    return &it->second;
  }
}

// Guard G statistics of the last orc_apply (test infrastructure; the
// definition the engine's per-dict replay measures, include/crdtm.h
// crdtm_ctx_guard_stats): Adds whose findInsertion walk ran, and those whose
// walk met a Tombstone above their timestamp as a raw `next` key.
struct GStats {
  uint64_t walked = 0, fail = 0;
  uint64_t reached = 0;  // ops whose path resolution reached their dict (update called the leaf function)
};
thread_local GStats g_gstats;

// findInsertion (src/Internal/Node.elm:93-104). Returns (leftKey, leftNode);
// after a tombstone skip leftKey != key(leftNode) (Appendix A.5).
std::pair<int64_t, Node*> findInsertion(int64_t ts, int64_t n, Node* node, Dict& c) {
  ++g_gstats.walked;
  bool gfail = false;
  auto done = [&](std::pair<int64_t, Node*> r) {
    if (gfail) ++g_gstats.fail;
    return r;
  };
  for (;;) {
    if (node->kind == ROOT || !node->has_next) return done({n, node});
    const int64_t k = node->next;
    auto it = c.find(k);
    if (it != c.end() && it->second.kind == TOMB && ts < k) gfail = true;  // (statistics only)
    Node* live = nextNode(node, c);
    if (!live) return done({n, node});
    if (ts > k) return done({n, node});
    n = k;
    node = live;
  }
}

// insert (src/Internal/Node.elm:125-135): no-op on a Tombstone parent.
void insert(int64_t ts, Node&& node, Node& parent) {
  if (parent.kind == TOMB) return;
  parent.children[ts] = std::move(node);
}

// addAfterHelp (src/Internal/Node.elm:56-90)
int addAfterHelp(const std::vector<int64_t>& p, int64_t ts, uint32_t val, int64_t prevTs, Node& parent) {
  if (child(ts, parent)) return N_ALREADY;
  Node* found = child(prevTs, parent);
  if (!found) return N_NOTFOUND;
  Dict& c = parent.children;  // parent is Root/Node here (update rejected Tombstones)
  auto [leftTs, left] = findInsertion(ts, prevTs, found, c);
  Node node;
  node.kind = NODE;
  node.val = val;
  node.path.assign(p.begin(), p.end() - 1);  // Array.slice 0 -1
  node.path.push_back(ts);                   // Array.push ts
  node.has_next = left->has_next;            // next left
  node.next = left->next;
  node.children = emptyChildren();
  // parent |> insert leftTs (updateNext ts left) |> insert ts node
  auto slot = c.find(leftTs);
  if (slot != c.end() && &slot->second == left) {
    left->has_next = true;  // updateNext in place: same value, same slot
    left->next = ts;
  } else {
    Node copy = *left;      // copy quirk: slot leftTs receives a copy of left (deep: Elm values are persistent)
    copy.has_next = true;
    copy.next = ts;
    insert(leftTs, std::move(copy), parent);
  }
  insert(ts, std::move(node), parent);
  return N_OK;
}

// deleteHelp (src/Internal/Node.elm:112-122)
int deleteHelp(int64_t ts, Node& parent) {
  Node* c = child(ts, parent);
  if (!c) return N_NOTFOUND;
  if (c->kind == NODE) {  // Tombstone p n: drop value and children
    c->kind = TOMB;
    c->val = 0;
    c->children.clear();
    return N_OK;
  }
  return N_ALREADY;
}

// update (src/Internal/Node.elm:138-163). Mutates in place; every error is
// returned before the leaf function mutates anything.
template <class F>
int update(F&& func, const int64_t* p, size_t len, Node& parent) {
  if (parent.kind == TOMB) return N_ALREADY;
  if (len == 0) return N_INVALID;
  if (len == 1) {
    ++g_gstats.reached;  // (statistics only)
    return func(p[0], parent);
  }
  Node* found = child(p[0], parent);
  if (!found) return N_INVALID;
  return update(func, p + 1, len - 1, *found);
}

// Operation a = Add Int (List Int) a | Delete (List Int) | Batch (List (Operation a))
// (src/Internal/Operation.elm:17-20)
enum OpKind : int { OP_ADD = 0, OP_DEL = 1, OP_BATCH = 2 };
struct Op {
  int kind = OP_BATCH;
  int64_t ts = 0;
  std::vector<int64_t> path;
  uint32_t val = 0;
  int64_t index = -1;       // position in the caller's flattened op array
  std::vector<Op> ops;      // Batch
};

// Timestamp.replicaId ts = ts // 2^32 (src/CRDTree/Timestamp.elm:16-18); Elm `//`
// on JS numbers is (a / b) | 0 — truncation toward zero, exact for |ts| < 2^53.
int64_t replicaId(int64_t ts) { return ts / 4294967296LL; }

// CRDTree record (src/CRDTree.elm:112-120)
struct Tree {
  Node root;
  int64_t timestamp = 0;
  std::vector<int64_t> cursor;
  std::vector<Op> operations;   // oldest-first here; Elm keeps newest-first (cons)
  std::map<int64_t, int64_t> replicas;
  bool last_is_batch = true;    // lastOperation: Batch list, or a single Add/Delete
  std::vector<Op> last;
  int64_t err_index = -1;
};

// Operation.toList (src/Internal/Operation.elm:58-68): a single Add/Delete is
// held as a one-element list with last_is_batch = false, so toList is the list.
std::vector<Op> toList(const std::vector<Op>& l) { return l; }

// init (src/CRDTree.elm:130-139); Node.root (src/Internal/Node.elm:41-43)
void initTree(Tree& t, int64_t replica) {
  t.root = Node();
  t.root.kind = ROOT;
  t.root.children = emptyChildren();
  t.timestamp = replica * 4294967296LL;  // replicaId * 2 ^ 32
  t.cursor = {0};
  t.operations.clear();
  t.replicas.clear();
  t.last_is_batch = true;
  t.last.clear();
}

int64_t treeId(const Tree& t) { return replicaId(t.timestamp); }  // id (src/CRDTree.elm:378-380)

// buildPath (src/CRDTree.elm:628-632)
std::vector<int64_t> buildPath(int64_t ts, const std::vector<int64_t>& path) {
  std::vector<int64_t> r;
  if (!path.empty()) r.assign(path.begin(), path.end() - 1);
  r.push_back(ts);
  return r;
}

// updateTree (src/CRDTree.elm:298-325)
int updateTree(const Op& op, const std::vector<int64_t>& path, int64_t ts, Tree& t, int nres) {
  switch (nres) {
    case N_OK:
      t.cursor = buildPath(ts, path);
      t.operations.push_back(op);
      t.last_is_batch = false;
      t.last.assign(1, op);
      t.replicas[replicaId(ts)] = ts;
      return T_OK;
    case N_ALREADY:
      t.last_is_batch = true;
      t.last.clear();
      return T_OK;
    case N_INVALID:
      t.err_index = op.index;
      return T_INVALID_PATH;
    default:
      t.err_index = op.index;
      return T_OPERATION_FAILED;
  }
}

int apply(const Op& op, Tree& t);

// batch (src/CRDTree.elm:224-232) with mergeOperations (:328-334) and
// Operation.merge = Batch (toList a ++ toList b) (src/Internal/Operation.elm:80-82)
int batch(const std::vector<Op>& ops, Tree& t) {
  t.last_is_batch = true;
  t.last.clear();
  for (const Op& o : ops) {
    std::vector<Op> prev = std::move(t.last);
    t.last.clear();
    int r = apply(o, t);
    if (r != T_OK) return r;
    // merge one.lastOperation two.lastOperation = Batch (toList one ++ toList two);
    // appended in place (the reference copies the accumulator: O(n^2), §6)
    std::vector<Op> merged = std::move(prev);
    for (auto& x : toList(t.last)) merged.push_back(std::move(x));
    t.last = std::move(merged);
    t.last_is_batch = true;
  }
  return T_OK;
}

// incrementTimestamp (src/CRDTree.elm:337-343)
void incrementTimestamp(int64_t ts, Tree& t) {
  if (replicaId(ts) == treeId(t)) t.timestamp = t.timestamp + 1;
}

// applyLocal (src/CRDTree.elm:275-295)
int applyLocal(const Op& op, Tree& t) {
  switch (op.kind) {
    case OP_ADD: {
      const int64_t ts = op.ts;
      const uint32_t val = op.val;
      const std::vector<int64_t>& p = op.path;
      int nres = update(
          [&](int64_t prevTs, Node& parent) { return addAfterHelp(p, ts, val, prevTs, parent); },
          p.data(), p.size(), t.root);
      int r = updateTree(op, p, ts, t, nres);
      if (r == T_OK) incrementTimestamp(ts, t);
      return r;
    }
    case OP_DEL: {
      // Operation.timestamp (Delete p) = List.reverse p |> List.head, default 0
      const int64_t ots = op.path.empty() ? 0 : op.path.back();
      int nres = update([&](int64_t k, Node& parent) { return deleteHelp(k, parent); }, op.path.data(),
                        op.path.size(), t.root);
      return updateTree(op, op.path, ots, t, nres);
    }
    default:
      return batch(op.ops, t);
  }
}

// apply (src/CRDTree.elm:265-269): applyLocal, then restore the caller's cursor
int apply(const Op& op, Tree& t) {
  std::vector<int64_t> saved = t.cursor;
  int r = applyLocal(op, t);
  if (r == T_OK) t.cursor = saved;
  return r;
}

// ---- canonical dumps (shared format with the product's crdtm_tree_canonical) ----

constexpr uint64_t FNV_OFF = 1469598103934665603ULL, FNV_PRIME = 1099511628211ULL;
struct Sink {
  std::vector<int64_t>* out;  // may be null: hash only
  uint64_t h = FNV_OFF;
  uint64_t n = 0;
  void put(int64_t w) {
    if (out) out->push_back(w);
    h ^= static_cast<uint64_t>(w);  // word-wise FNV-1a over 64-bit words
    h *= FNV_PRIME;
    ++n;
  }
};

// Structure: every dict entry (incl. tombstones, sentinels, orphans), ascending keys, DFS.
void dumpDict(const Dict& d, int64_t depth, Sink& s) {
  for (const auto& [key, n] : d) {
    s.put(depth);
    s.put(key);
    s.put(n.kind);
    s.put(n.has_next ? 1 : 0);
    s.put(n.has_next ? n.next : 0);
    s.put(n.kind == NODE ? static_cast<int64_t>(n.val) : 0);
    s.put(static_cast<int64_t>(n.path.size()));
    for (int64_t x : n.path) s.put(x);
    if (n.kind == NODE) dumpDict(n.children, depth + 1, s);
  }
}

// Visible document order: from sentinel 0 follow nextNode (src/Internal/Node.elm:206-228),
// recursing into each live node's children (pre-order).
void dumpVisible(const Dict& cd, int64_t depth, Sink& s) {
  Dict& c = const_cast<Dict&>(cd);
  auto it = c.find(0);
  if (it == c.end()) return;
  Node* cur = &it->second;
  for (;;) {
    Node* nx = nextNode(cur, c);
    if (!nx) break;
    s.put(depth);
    s.put(static_cast<int64_t>(nx->val));
    s.put(static_cast<int64_t>(nx->path.size()));
    for (int64_t x : nx->path) s.put(x);
    dumpVisible(nx->children, depth + 1, s);
    cur = nx;
  }
}

Op makeOp(uint8_t kind, int64_t ts, const int64_t* path, uint32_t plen, uint32_t val, int64_t index) {
  Op o;
  o.kind = kind == 0 ? OP_ADD : OP_DEL;
  o.ts = kind == 0 ? ts : 0;
  o.path.assign(path, path + plen);
  o.val = kind == 0 ? val : 0;
  o.index = index;
  return o;
}

Node* descendant(const int64_t* p, size_t len, Node& n) {  // src/Internal/Node.elm:289-299
  if (len == 0) return nullptr;
  Node* c = child(p[0], n);
  if (len == 1 || !c) return c;
  return descendant(p + 1, len - 1, *c);
}

}  // namespace

extern "C" {

struct orc_tree { Tree t; };

orc_tree* orc_init(int64_t replica) {
  auto* o = new orc_tree;
  initTree(o->t, replica);
  return o;
}
orc_tree* orc_clone(const orc_tree* o) { return new orc_tree(*o); }
void orc_free(orc_tree* o) { delete o; }

// apply (op | Batch ops) to the tree. Ops arrive flattened (kind 0 = Add,
// 1 = Delete); is_batch selects `apply (Batch ops)` vs `apply op` (n_ops == 1).
// local != 0 uses applyLocal (cursor not restored; the local add/addAfter path).
// Returns CRDTree.Error code (0 = Ok); *err_index = flattened index of the
// failing op. On error the tree is unchanged (Elm persistence).
int orc_apply(orc_tree* o, int is_batch, int local, uint64_t n_ops, const uint8_t* kind, const int64_t* ts,
              const uint32_t* path_off, const int64_t* path, const uint32_t* val, int64_t* err_index) {
  Op top;
  if (is_batch) {
    top.kind = OP_BATCH;
    top.ops.reserve(n_ops);
    for (uint64_t i = 0; i < n_ops; ++i)
      top.ops.push_back(makeOp(kind[i], ts[i], path + path_off[i], path_off[i + 1] - path_off[i], val[i],
                               static_cast<int64_t>(i)));
  } else {
    top = makeOp(kind[0], ts[0], path + path_off[0], path_off[1] - path_off[0], val[0], 0);
  }
  Tree work = o->t;  // Elm: the caller still holds the old tree on Err
  work.err_index = -1;
  g_gstats = GStats{};
  int r = local ? applyLocal(top, work) : apply(top, work);
  if (err_index) *err_index = work.err_index;
  if (r == T_OK) o->t = std::move(work);
  return r;
}

// guard G statistics of the last orc_apply: out[0] Adds whose findInsertion
// walk ran, out[1] those that met a Tombstone above their timestamp, out[2]
// the ops whose path resolution reached their dict (no Tombstone on the way,
// no missing child)
void orc_guard_stats(uint64_t* out) {
  out[0] = g_gstats.walked;
  out[1] = g_gstats.fail;
  out[2] = g_gstats.reached;
}

int64_t orc_timestamp(const orc_tree* o) { return o->t.timestamp; }
void orc_set_timestamp(orc_tree* o, int64_t ts) { o->t.timestamp = ts; }

uint64_t orc_cursor(const orc_tree* o, int64_t* out, uint64_t cap) {
  for (uint64_t i = 0; i < o->t.cursor.size() && i < cap; ++i) out[i] = o->t.cursor[i];
  return o->t.cursor.size();
}
void orc_set_cursor(orc_tree* o, const int64_t* p, uint64_t n) { o->t.cursor.assign(p, p + n); }

uint64_t orc_replicas(const orc_tree* o, int64_t* ids, int64_t* tss, uint64_t cap) {
  uint64_t i = 0;
  for (const auto& [k, v] : o->t.replicas) {
    if (i < cap) { ids[i] = k; tss[i] = v; }
    ++i;
  }
  return i;
}

// Op list export (operations log oldest-first, or lastOperation's list).
// which: 0 = operations log, 1 = lastOperation. Returns count; fills arrays
// when non-null (path buffer sized by *path_total on a first call).
uint64_t orc_ops(const orc_tree* o, int which, uint8_t* kind, int64_t* ts, uint32_t* path_off, int64_t* path,
                 uint32_t* val, uint64_t* path_total, int* is_batch) {
  const std::vector<Op>& l = which == 0 ? o->t.operations : o->t.last;
  if (is_batch) *is_batch = which == 0 ? 1 : (o->t.last_is_batch ? 1 : 0);
  uint64_t pt = 0;
  for (uint64_t i = 0; i < l.size(); ++i) {
    if (kind) kind[i] = static_cast<uint8_t>(l[i].kind);
    if (ts) ts[i] = l[i].ts;
    if (val) val[i] = l[i].val;
    if (path_off) path_off[i] = static_cast<uint32_t>(pt);
    if (path) {
      for (int64_t x : l[i].path) path[pt++] = x;
    } else {
      pt += l[i].path.size();
    }
  }
  if (path_off) path_off[l.size()] = static_cast<uint32_t>(pt);
  if (path_total) *path_total = pt;
  return l.size();
}

// Canonical dumps. which: 0 = structure, 1 = visible order. If out is null
// only the hash/word count are produced. Returns the word count.
uint64_t orc_canonical(const orc_tree* o, int which, int64_t* out, uint64_t cap, uint64_t* hash) {
  std::vector<int64_t> buf;
  Sink s{out ? &buf : nullptr};
  if (which == 0) dumpDict(o->t.root.children, 0, s);
  else dumpVisible(o->t.root.children, 0, s);
  if (out) for (uint64_t i = 0; i < buf.size() && i < cap; ++i) out[i] = buf[i];
  if (hash) *hash = s.h;
  return s.n;
}

// get path tree |> value (CRDTree.getValue, src/CRDTree.elm:486-488).
// Returns 1 = Just (value in *val), 0 = Nothing (missing or tombstone).
// *exists = 1 if `get` found a node (Node or Tombstone).
int orc_get_value(orc_tree* o, const int64_t* p, uint64_t n, uint32_t* val, int* exists) {
  Node* d = descendant(p, n, o->t.root);
  if (exists) *exists = d ? 1 : 0;
  if (!d || d->kind != NODE) return 0;
  if (val) *val = d->val;
  return 1;
}

// Node.path of the node at `p` (for the `delete` local cursor logic and tests).
uint64_t orc_get_path(orc_tree* o, const int64_t* p, uint64_t n, int64_t* out, uint64_t cap) {
  Node* d = descendant(p, n, o->t.root);
  if (!d) return UINT64_MAX;
  for (uint64_t i = 0; i < d->path.size() && i < cap; ++i) out[i] = d->path[i];
  return d->path.size();
}

}  // extern "C"

// ---- traversal (src/CRDTree.elm:421-625, src/CRDTree/Node.elm:96-174) ----
// Results are node descriptors written as words: kind (1 Node, 2 Tombstone,
// 3 Root), value handle (Node; else 0), has_next, next, path length, path.

static void putNode(const Node* d, std::vector<int64_t>& out) {
  out.push_back(d->kind == ROOT ? 3 : d->kind);
  out.push_back(d->kind == NODE ? d->val : 0);
  out.push_back(d->kind != ROOT && d->has_next ? 1 : 0);
  out.push_back(d->kind != ROOT && d->has_next ? d->next : 0);
  out.push_back(static_cast<int64_t>(d->path.size()));
  for (int64_t k : d->path) out.push_back(k);
}

static uint64_t emit(const std::vector<int64_t>& w, int64_t* out, uint64_t cap) {
  for (uint64_t i = 0; out && i < w.size() && i < cap; ++i) out[i] = w[i];
  return w.size();
}

// parent (src/CRDTree.elm:425-441): path minus its last key; [] -> the root
static Node* parentOf(Tree& t, Node* node) {
  std::vector<int64_t> pp = node->path;
  if (!pp.empty()) pp.pop_back();  // Array.slice 0 -1
  if (pp.empty()) return &t.root;
  return descendant(pp.data(), pp.size(), t.root);
}

static Dict kEmpty;
static Dict& childrenOf(Node* n) { return n->kind == TOMB ? kEmpty : n->children; }  // src/Internal/Node.elm:231-241

// next (src/CRDTree.elm:560-566)
static Node* nextOf(Tree& t, Node* node) {
  Node* par = parentOf(t, node);
  if (!par) return nullptr;
  return nextNode(node, childrenOf(par));
}

// Elm structural equality on Node values
static bool nodeEq(const Node& a, const Node& b) {
  if (a.kind != b.kind || a.path != b.path) return false;
  if (a.kind == NODE && a.val != b.val) return false;
  const bool an = a.kind != ROOT && a.has_next, bn = b.kind != ROOT && b.has_next;
  if (an != bn || (an && a.next != b.next)) return false;
  if (a.children.size() != b.children.size()) return false;
  for (auto ia = a.children.begin(), ib = b.children.begin(); ia != a.children.end(); ++ia, ++ib)
    if (ia->first != ib->first || !nodeEq(ia->second, ib->second)) return false;
  return true;
}

// prev (src/CRDTree.elm:569-575): Node.find over the parent's chain from its
// sentinel, Tombstones included (findHelp, src/Internal/Node.elm:170-182)
static Node* prevOf(Tree& t, Node* node) {
  Node* par = parentOf(t, node);
  if (!par) return nullptr;
  Dict& c = childrenOf(par);
  auto it = c.find(0);
  if (it == c.end()) return nullptr;
  Node* left = &it->second;
  for (;;) {
    if (left->kind == ROOT || !left->has_next) return nullptr;
    auto jt = c.find(left->next);
    if (jt == c.end()) return nullptr;
    Node* n = &jt->second;
    Node* nn = nextOf(t, n);
    if (nn && nodeEq(*nn, *node)) return n;
    left = n;
  }
}

// head (src/CRDTree/Node.elm:165-167): first live child
static Node* headOf(Node* node) {
  Dict& c = childrenOf(node);
  auto it = c.find(0);
  if (it == c.end()) return nullptr;
  return nextNode(&it->second, c);
}

// walkHelp (src/CRDTree.elm:602-625) with a function that always Takes
static void walkHelp(Node* left, Dict& siblings, std::vector<int64_t>& out) {
  for (;;) {
    Node* node = nextNode(left, siblings);
    if (!node) return;
    putNode(node, out);
    Node* h = headOf(node);
    if (h) walkHelp(h, childrenOf(node), out);
    left = node;
  }
}

extern "C" {

// get (src/CRDTree.elm:468-470) -> one descriptor, or 0 words (Nothing)
uint64_t orc_node_get(orc_tree* o, const int64_t* p, uint64_t n, int64_t* out, uint64_t cap) {
  std::vector<int64_t> w;
  Node* d = descendant(p, n, o->t.root);
  if (d) putNode(d, w);
  return emit(w, out, cap);
}

// which: 0 parent, 1 next, 2 prev, 3 CRDTree.Node.children (live, chain order),
// 4 walk from the node (Just node), 5 walk from the start (Nothing; p ignored)
uint64_t orc_node_query(orc_tree* o, int which, const int64_t* p, uint64_t n, int64_t* out, uint64_t cap) {
  std::vector<int64_t> w;
  Tree& t = o->t;
  Node* d = which == 5 ? nullptr : (n == 0 ? &t.root : descendant(p, n, t.root));
  if (which != 5 && !d) return emit(w, out, cap);
  Node* r = nullptr;
  switch (which) {
    case 0: r = parentOf(t, d); break;
    case 1: r = nextOf(t, d); break;
    case 2: r = prevOf(t, d); break;
    case 3: {
      Dict& c = childrenOf(d);
      auto it = c.find(0);
      for (Node* x = it == c.end() ? nullptr : nextNode(&it->second, c); x; x = nextNode(x, c)) putNode(x, w);
      return emit(w, out, cap);
    }
    case 4: {
      Node* par = parentOf(t, d);
      if (par) walkHelp(d, childrenOf(par), w);
      return emit(w, out, cap);
    }
    case 5: {
      Node* h = headOf(&t.root);
      if (h) {
        Node* par = parentOf(t, h);
        if (par) walkHelp(h, childrenOf(par), w);
      }
      return emit(w, out, cap);
    }
  }
  if (r) putNode(r, w);
  return emit(w, out, cap);
}

}  // extern "C"

extern "C" {

// lastOperation := Batch [] (the reset `batch` performs, src/CRDTree.elm:231)
void orc_reset_last(orc_tree* o) { o->t.last_is_batch = true; o->t.last.clear(); }

// Append lastOperation of `other` to `o`'s lastOperation (mergeOperations for
// a Python-side `batch` of local functions, src/CRDTree.elm:328-334).
void orc_merge_last(orc_tree* o, const orc_tree* prev) {
  std::vector<Op> merged = prev->t.last;
  for (auto& x : o->t.last) merged.push_back(x);
  o->t.last = std::move(merged);
  o->t.last_is_batch = true;
}

}  // extern "C"

// ---- flat fast restatement (test infrastructure) ----
// The same findInsertion / addAfterHelp semantics (src/Internal/Node.elm:56-104)
// specialised to an Adds-only batch on a fresh tree whose paths all have
// length 1 (one dict, no Tombstone besides the sentinel, so no copy quirk):
// the dict is an array of keys in ascending order with a `next` link per
// key. Pinned against orc_apply by tests/test_oracle_kat.py. Returns 0 (Ok),
// 3 (OperationFailed) with *err_index, or -1 when the batch is outside the
// specialisation (a Delete, a path of length != 1). hash[0..1] / words[0..1]
// receive the canonical structure and visible-order digests (orc_canonical).
//
// Two ways to run findInsertion's walk (:93-104), same `next` links:
//  * literal (orc_flat_replay_literal): follow `next` from the anchor while
//    the inserted key is below the next key. A walk passes every larger key
//    after its anchor, so a low replica id's Add in a long document walks
//    ~10^4-10^5 nodes: config 3's 10M ops take hours;
//  * searched (orc_flat_replay): the same stop node found in O(log n). The
//    loop stops at the last node u after the anchor such that every node
//    after the anchor up to u has a key above x (keys are distinct: `made`),
//    i.e. u = the node before the first node after the anchor whose key is
//    below x, or the list's last node when there is none. A treap over the
//    list order with the smallest key per subtree finds that first node
//    (climb from the anchor, descend into the first subtree whose minimum is
//    below x). Used for full-size parity of config 3; pinned against the
//    literal walk by tests/test_oracle_flat.py.
namespace {
struct ListTreap {  // in-order = the dict's `next` order; ids = key slots (slot order = key order)
  static constexpr uint32_t NIL = 0xFFFFFFFFu;
  std::vector<uint32_t> L, R, P, mn;
  uint32_t root = NIL;
  explicit ListTreap(size_t k) : L(k, NIL), R(k, NIL), P(k, NIL), mn(k, NIL) {}
  static uint64_t pri(uint32_t v) {
    uint64_t z = v + 0x9E3779B97F4A7C15ULL;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
  }
  uint32_t submin(uint32_t t) const { return t == NIL ? NIL : mn[t]; }
  void pull(uint32_t t) { mn[t] = std::min(t, std::min(submin(L[t]), submin(R[t]))); }
  // the first node at or after the in-order start of subtree t with id < x
  uint32_t leftmost_less(uint32_t t, uint32_t x) const {
    for (;;) {
      if (L[t] != NIL && mn[L[t]] < x) t = L[t];
      else if (t < x) return t;
      else t = R[t];
    }
  }
  // the first node after a (in-order) with id < x, NIL if none
  uint32_t first_after_less(uint32_t a, uint32_t x) const {
    if (R[a] != NIL && mn[R[a]] < x) return leftmost_less(R[a], x);
    for (uint32_t c = a; P[c] != NIL; c = P[c]) {
      const uint32_t p = P[c];
      if (L[p] != c) continue;  // c was p's right child: p comes before
      if (p < x) return p;
      if (R[p] != NIL && mn[R[p]] < x) return leftmost_less(R[p], x);
    }
    return NIL;
  }
  uint32_t pred(uint32_t b) const {
    if (L[b] != NIL) {
      uint32_t t = L[b];
      while (R[t] != NIL) t = R[t];
      return t;
    }
    uint32_t c = b;
    while (P[c] != NIL && L[P[c]] == c) c = P[c];
    return P[c];
  }
  uint32_t last() const {
    uint32_t t = root;
    while (R[t] != NIL) t = R[t];
    return t;
  }
  void rotate_up(uint32_t y) {  // y takes its parent's place
    const uint32_t p = P[y], g = P[p];
    if (L[p] == y) {
      L[p] = R[y];
      if (R[y] != NIL) P[R[y]] = p;
      R[y] = p;
    } else {
      R[p] = L[y];
      if (L[y] != NIL) P[L[y]] = p;
      L[y] = p;
    }
    P[p] = y;
    P[y] = g;
    if (g == NIL) root = y;
    else if (L[g] == p) L[g] = y;
    else R[g] = y;
    pull(p);
    pull(y);
  }
  void insert_first(uint32_t y) {
    root = y;
    mn[y] = y;
  }
  // y right after u in the order
  void insert_after(uint32_t u, uint32_t y) {
    uint32_t at = u;
    bool left = false;
    if (R[u] != NIL) {
      at = R[u];
      while (L[at] != NIL) at = L[at];
      left = true;
    }
    (left ? L[at] : R[at]) = y;
    P[y] = at;
    mn[y] = y;
    for (uint32_t t = at; t != NIL && mn[t] > y; t = P[t]) mn[t] = y;
    while (P[y] != NIL && pri(y) > pri(P[y])) rotate_up(y);
  }
};

int flat_replay(bool searched, uint64_t n, const uint8_t* kind, const int64_t* ts, const uint32_t* path_off,
                const int64_t* path, const uint32_t* val, int64_t* err_index, uint64_t* hash, uint64_t* words,
                uint64_t* n_applied);
}  // namespace

extern "C" int orc_flat_replay(uint64_t n, const uint8_t* kind, const int64_t* ts, const uint32_t* path_off,
                               const int64_t* path, const uint32_t* val, int64_t* err_index, uint64_t* hash,
                               uint64_t* words, uint64_t* n_applied) {
  return flat_replay(true, n, kind, ts, path_off, path, val, err_index, hash, words, n_applied);
}

extern "C" int orc_flat_replay_literal(uint64_t n, const uint8_t* kind, const int64_t* ts, const uint32_t* path_off,
                                       const int64_t* path, const uint32_t* val, int64_t* err_index, uint64_t* hash,
                                       uint64_t* words, uint64_t* n_applied) {
  return flat_replay(false, n, kind, ts, path_off, path, val, err_index, hash, words, n_applied);
}

namespace {
int flat_replay(bool searched, uint64_t n, const uint8_t* kind, const int64_t* ts, const uint32_t* path_off,
                const int64_t* path, const uint32_t* val, int64_t* err_index, uint64_t* hash, uint64_t* words,
                uint64_t* n_applied) {
  std::vector<int64_t> keys;
  keys.reserve(n + 1);
  keys.push_back(0);
  for (uint64_t i = 0; i < n; ++i) {
    if (kind[i] != 0 || path_off[i + 1] - path_off[i] != 1) return -1;
    keys.push_back(ts[i]);
  }
  std::sort(keys.begin(), keys.end());
  keys.erase(std::unique(keys.begin(), keys.end()), keys.end());
  const size_t K = keys.size();
  auto slot = [&](int64_t k) -> int64_t {
    auto it = std::lower_bound(keys.begin(), keys.end(), k);
    return (it != keys.end() && *it == k) ? it - keys.begin() : -1;
  };
  constexpr uint32_t NIL = 0xFFFFFFFFu;
  std::vector<uint32_t> nxt(K, NIL), v(K, 0);
  std::vector<uint8_t> made(K, 0);
  const int64_t z = slot(0);
  made[z] = 1;  // the sentinel 0 -> Tombstone [] Nothing
  ListTreap tr(searched ? K : 0);
  if (searched) tr.insert_first(static_cast<uint32_t>(z));
  uint64_t applied = 0;
  for (uint64_t i = 0; i < n; ++i) {
    const int64_t x = slot(ts[i]);  // always found
    if (made[x]) continue;          // child ts parent exists: AlreadyApplied (the sentinel too)
    const int64_t a = slot(path[path_off[i]]);
    if (a < 0 || !made[a]) {        // anchor missing: NotFound -> OperationFailed
      *err_index = static_cast<int64_t>(i);
      return 3;
    }
    // findInsertion: slot order is key order, and no node but the sentinel is a Tombstone
    uint32_t node = static_cast<uint32_t>(a);
    if (searched) {
      const uint32_t b = tr.first_after_less(node, static_cast<uint32_t>(x));
      node = b == NIL ? tr.last() : tr.pred(b);
      tr.insert_after(node, static_cast<uint32_t>(x));
    } else {
      for (;;) {
        const uint32_t rn = nxt[node];
        if (rn == NIL || x > static_cast<int64_t>(rn)) break;
        node = rn;
      }
    }
    nxt[x] = nxt[node];
    nxt[node] = static_cast<uint32_t>(x);
    v[x] = val[i];
    made[x] = 1;
    ++applied;
  }
  *n_applied = applied;
  // canonical dumps, same words as dumpDict / dumpVisible
  Sink s0{nullptr}, s1{nullptr};
  for (size_t q = 0; q < K; ++q) {
    if (!made[q]) continue;
    const bool hn = nxt[q] != NIL;
    s0.put(0);
    s0.put(keys[q]);
    s0.put(static_cast<int64_t>(q) == z ? TOMB : NODE);
    s0.put(hn ? 1 : 0);
    s0.put(hn ? keys[nxt[q]] : 0);
    s0.put(static_cast<int64_t>(q) == z ? 0 : static_cast<int64_t>(v[q]));
    if (static_cast<int64_t>(q) == z) {
      s0.put(0);
      continue;
    }
    s0.put(1);
    s0.put(keys[q]);
    // its children: emptyChildren = {0: Tombstone [] Nothing}
    s0.put(1); s0.put(0); s0.put(TOMB); s0.put(0); s0.put(0); s0.put(0); s0.put(0);
  }
  for (uint32_t q = nxt[z]; q != NIL; q = nxt[q]) {
    s1.put(0);
    s1.put(static_cast<int64_t>(v[q]));
    s1.put(1);
    s1.put(keys[q]);
  }
  hash[0] = s0.h;
  hash[1] = s1.h;
  words[0] = s0.n;
  words[1] = s1.n;
  return 0;
}
}  // namespace

// ---- full-size property check of a flat merge (test infrastructure) ----
// For an Adds-only batch with paths of length 1 on a fresh tree, every
// findInsertion walk (src/Internal/Node.elm:93-104) skips only keys larger
// than the inserted one, and a later insertion lands between an anchor and
// x only if it is larger than x (induction on the batch); so in the final
// document order: (1) every applied key appears once, (2) each key comes
// after its anchor, (3) every key strictly between the anchor and the key
// is larger than the key, i.e. the nearest smaller key to its left is at or
// before the anchor (the sentinel sits before position 0). O(n log n).
// Returns the number of violations (0 = the order has all three properties).
extern "C" uint64_t orc_flat_check(uint64_t n_doc, const int64_t* doc_keys, uint64_t n, const int64_t* ts,
                                   const uint32_t* path_off, const int64_t* path) {
  std::vector<std::pair<int64_t, int64_t>> kp(n_doc);
  for (uint64_t p = 0; p < n_doc; ++p) kp[p] = {doc_keys[p], static_cast<int64_t>(p)};
  std::sort(kp.begin(), kp.end());
  uint64_t bad = 0;
  for (uint64_t p = 1; p < n_doc; ++p)
    if (kp[p].first == kp[p - 1].first) ++bad;  // a key twice
  auto pos = [&](int64_t k) -> int64_t {
    auto it = std::lower_bound(kp.begin(), kp.end(), std::make_pair(k, INT64_MIN));
    return (it != kp.end() && it->first == k) ? it->second : -2;
  };
  std::vector<int64_t> ps(n_doc), st;  // nearest smaller key to the left (monotonic stack)
  st.reserve(1024);
  for (uint64_t p = 0; p < n_doc; ++p) {
    while (!st.empty() && doc_keys[st.back()] > doc_keys[p]) st.pop_back();
    ps[p] = st.empty() ? -1 : st.back();
    st.push_back(static_cast<int64_t>(p));
  }
  uint64_t seen = 0;
  for (uint64_t i = 0; i < n; ++i) {
    if (path_off[i + 1] - path_off[i] != 1) return ~0ULL;
    const int64_t px = pos(ts[i]);
    if (px < 0) {
      ++bad;  // an applied key missing from the document
      continue;
    }
    ++seen;
    const int64_t a = path[path_off[i]];
    const int64_t pa = a == 0 ? -1 : pos(a);
    if (pa == -2 || pa >= px || ps[px] > pa) ++bad;
  }
  if (seen != n_doc) ++bad;
  return bad;
}

// ---- many independent documents (test infrastructure; config 5) ----
// Document d = ops [doc_off[d], doc_off[d+1]) applied as `apply (Batch ops_d)`
// to a fresh `init replica` (src/CRDTree.elm:130-139, :265-269), exactly like
// orc_init + orc_apply + orc_canonical(which = 1) + orc_timestamp per document,
// without a host round trip per document. Per-document outputs: error code,
// local err index (-1), visible-order digest and word count, final timestamp.
extern "C" void orc_forest_apply(uint64_t n_docs, const uint32_t* doc_off, int64_t replica, const uint8_t* kind,
                                 const int64_t* ts, const uint32_t* path_off, const int64_t* path,
                                 const uint32_t* val, int32_t* code, int64_t* err, uint64_t* vhash,
                                 uint64_t* vwords, int64_t* tstamp) {
  for (uint64_t d = 0; d < n_docs; ++d) {
    const uint32_t a = doc_off[d], b = doc_off[d + 1];
    Tree t;
    initTree(t, replica);
    Op top;
    top.kind = OP_BATCH;
    top.ops.reserve(b - a);
    for (uint32_t i = a; i < b; ++i)
      top.ops.push_back(makeOp(kind[i], ts[i], path + path_off[i], path_off[i + 1] - path_off[i], val[i],
                               static_cast<int64_t>(i - a)));
    t.err_index = -1;
    const int r = apply(top, t);
    code[d] = r;
    err[d] = r == T_OK ? -1 : t.err_index;
    Sink s{nullptr};
    if (r == T_OK) dumpVisible(t.root.children, 0, s);
    vhash[d] = s.h;
    vwords[d] = s.n;
    tstamp[d] = t.timestamp;
  }
}
