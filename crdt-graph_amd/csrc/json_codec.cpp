// json_codec.cpp — the reference's wire format, native.
//
// CRDTree.Operation.encoder / decoder (src/CRDTree/Operation.elm:109-159):
//   Add    -> {"op":"add","path":[int..],"ts":int,"val":V}
//   Delete -> {"op":"del","path":[int..]}
//   Batch  -> {"op":"batch","ops":[..]}          unknown "op" -> Batch []
// Bytes follow `Json.Encode.encode 0`, i.e. JSON.stringify without spaces
// (SURVEY.md A.10). Values are opaque to the merge; the decoder keeps each as
// the text JSON.stringify(JSON.parse(v)) would give (the Decode.value /
// Encode.value round trip), so re-encoding is byte-exact: numbers in
// ECMAScript Number::toString form, strings with JSON.stringify's escapes
// (lone surrogates as lower-case \udxxx), object keys in JS property order
// (array-index keys ascending, then insertion order; duplicates keep the first
// position and the last value).

#include <algorithm>
#include <charconv>
#include <cmath>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <string>
#include <utility>
#include <vector>

#include "../../include/crdtm.h"

namespace {

struct Parser {
  const char* s;
  size_t n;
  size_t i = 0;
  bool ok = true;
  int depth = 0;

  void ws() {
    while (i < n && (s[i] == ' ' || s[i] == '\t' || s[i] == '\n' || s[i] == '\r')) ++i;
  }
  bool eat(char c) {
    ws();
    if (i < n && s[i] == c) { ++i; return true; }
    return false;
  }
  void fail() { ok = false; }
};

// ---- strings: decode to UTF-16 code units (JS string semantics) ----
bool decodeUtf8(const char* s, size_t n, size_t& i, uint32_t& cp) {
  const unsigned char c = static_cast<unsigned char>(s[i]);
  if (c < 0x80) { cp = c; ++i; return true; }
  int len;
  if ((c & 0xE0) == 0xC0) { len = 2; cp = c & 0x1F; }
  else if ((c & 0xF0) == 0xE0) { len = 3; cp = c & 0x0F; }
  else if ((c & 0xF8) == 0xF0) { len = 4; cp = c & 0x07; }
  else return false;
  if (i + len > n) return false;
  for (int k = 1; k < len; ++k) {
    const unsigned char d = static_cast<unsigned char>(s[i + k]);
    if ((d & 0xC0) != 0x80) return false;
    cp = (cp << 6) | (d & 0x3F);
  }
  if ((len == 2 && cp < 0x80) || (len == 3 && cp < 0x800) || (len == 4 && (cp < 0x10000 || cp > 0x10FFFF)) ||
      (cp >= 0xD800 && cp <= 0xDFFF))
    return false;
  i += len;
  return true;
}

int hexv(char c) {
  if (c >= '0' && c <= '9') return c - '0';
  if (c >= 'a' && c <= 'f') return c - 'a' + 10;
  if (c >= 'A' && c <= 'F') return c - 'A' + 10;
  return -1;
}

bool parseString(Parser& p, std::u16string& out) {
  p.ws();
  if (p.i >= p.n || p.s[p.i] != '"') return false;
  ++p.i;
  out.clear();
  while (p.i < p.n) {
    const char c = p.s[p.i];
    if (c == '"') { ++p.i; return true; }
    if (static_cast<unsigned char>(c) < 0x20) return false;
    if (c == '\\') {
      if (p.i + 1 >= p.n) return false;
      const char e = p.s[p.i + 1];
      p.i += 2;
      switch (e) {
        case '"': out.push_back(u'"'); break;
        case '\\': out.push_back(u'\\'); break;
        case '/': out.push_back(u'/'); break;
        case 'b': out.push_back(u'\b'); break;
        case 'f': out.push_back(u'\f'); break;
        case 'n': out.push_back(u'\n'); break;
        case 'r': out.push_back(u'\r'); break;
        case 't': out.push_back(u'\t'); break;
        case 'u': {
          if (p.i + 4 > p.n) return false;
          int v = 0;
          for (int k = 0; k < 4; ++k) {
            const int h = hexv(p.s[p.i + k]);
            if (h < 0) return false;
            v = v * 16 + h;
          }
          p.i += 4;
          out.push_back(static_cast<char16_t>(v));
          break;
        }
        default: return false;
      }
      continue;
    }
    uint32_t cp;
    if (!decodeUtf8(p.s, p.n, p.i, cp)) return false;
    if (cp >= 0x10000) {
      cp -= 0x10000;
      out.push_back(static_cast<char16_t>(0xD800 + (cp >> 10)));
      out.push_back(static_cast<char16_t>(0xDC00 + (cp & 0x3FF)));
    } else {
      out.push_back(static_cast<char16_t>(cp));
    }
  }
  return false;
}

void putUtf8(std::string& o, uint32_t cp) {
  if (cp < 0x80) o.push_back(static_cast<char>(cp));
  else if (cp < 0x800) {
    o.push_back(static_cast<char>(0xC0 | (cp >> 6)));
    o.push_back(static_cast<char>(0x80 | (cp & 0x3F)));
  } else if (cp < 0x10000) {
    o.push_back(static_cast<char>(0xE0 | (cp >> 12)));
    o.push_back(static_cast<char>(0x80 | ((cp >> 6) & 0x3F)));
    o.push_back(static_cast<char>(0x80 | (cp & 0x3F)));
  } else {
    o.push_back(static_cast<char>(0xF0 | (cp >> 18)));
    o.push_back(static_cast<char>(0x80 | ((cp >> 12) & 0x3F)));
    o.push_back(static_cast<char>(0x80 | ((cp >> 6) & 0x3F)));
    o.push_back(static_cast<char>(0x80 | (cp & 0x3F)));
  }
}

// JSON.stringify(string) — ES2019 well-formed JSON.stringify (QuoteJSONString)
void quote(std::string& o, const std::u16string& u) {
  static const char* hx = "0123456789abcdef";
  o.push_back('"');
  for (size_t k = 0; k < u.size(); ++k) {
    const char16_t c = u[k];
    switch (c) {
      case u'"': o += "\\\""; continue;
      case u'\\': o += "\\\\"; continue;
      case u'\b': o += "\\b"; continue;
      case u'\f': o += "\\f"; continue;
      case u'\n': o += "\\n"; continue;
      case u'\r': o += "\\r"; continue;
      case u'\t': o += "\\t"; continue;
      default: break;
    }
    if (c < 0x20) {
      o += "\\u00";
      o.push_back(hx[(c >> 4) & 0xF]);
      o.push_back(hx[c & 0xF]);
    } else if (c >= 0xD800 && c <= 0xDBFF && k + 1 < u.size() && u[k + 1] >= 0xDC00 && u[k + 1] <= 0xDFFF) {
      putUtf8(o, 0x10000 + ((static_cast<uint32_t>(c) - 0xD800) << 10) + (u[k + 1] - 0xDC00));
      ++k;
    } else if (c >= 0xD800 && c <= 0xDFFF) {
      o += "\\u";
      for (int sh = 12; sh >= 0; sh -= 4) o.push_back(hx[(c >> sh) & 0xF]);
    } else {
      putUtf8(o, c);
    }
  }
  o.push_back('"');
}

// ---- numbers: ECMAScript Number::toString(x) ----
void jsNumber(std::string& o, double v) {
  if (v == 0) { o.push_back('0'); return; }  // also -0
  if (std::isnan(v) || std::isinf(v)) { o += "null"; return; }  // JSON.stringify(Infinity) = "null"
  if (v < 0) { o.push_back('-'); v = -v; }
  char buf[64];
  auto r = std::to_chars(buf, buf + sizeof(buf), v, std::chars_format::scientific);  // shortest round trip
  std::string sci(buf, r.ptr);
  const size_t epos = sci.find('e');
  std::string mant = sci.substr(0, epos);
  const int e10 = std::atoi(sci.c_str() + epos + 1);
  std::string digits;
  for (char c : mant)
    if (c != '.') digits.push_back(c);
  while (digits.size() > 1 && digits.back() == '0') digits.pop_back();
  const int k = static_cast<int>(digits.size());
  const int nexp = e10 + 1;  // value = 0.d1..dk * 10^nexp
  if (k <= nexp && nexp <= 21) {
    o += digits;
    o.append(static_cast<size_t>(nexp - k), '0');
  } else if (0 < nexp && nexp <= 21) {
    o += digits.substr(0, static_cast<size_t>(nexp));
    o.push_back('.');
    o += digits.substr(static_cast<size_t>(nexp));
  } else if (-6 < nexp && nexp <= 0) {
    o += "0.";
    o.append(static_cast<size_t>(-nexp), '0');
    o += digits;
  } else {
    o.push_back(digits[0]);
    if (k > 1) {
      o.push_back('.');
      o += digits.substr(1);
    }
    o.push_back('e');
    const int ex = nexp - 1;
    o.push_back(ex >= 0 ? '+' : '-');
    o += std::to_string(ex >= 0 ? ex : -ex);
  }
}

bool parseNumber(Parser& p, double& v, bool& integral_exact, long long& iv) {
  p.ws();
  const size_t b = p.i;
  if (p.i < p.n && p.s[p.i] == '-') ++p.i;
  if (p.i >= p.n) return false;
  if (p.s[p.i] == '0') ++p.i;
  else if (p.s[p.i] >= '1' && p.s[p.i] <= '9') while (p.i < p.n && p.s[p.i] >= '0' && p.s[p.i] <= '9') ++p.i;
  else return false;
  bool plain = true;
  if (p.i < p.n && p.s[p.i] == '.') {
    plain = false;
    ++p.i;
    if (p.i >= p.n || p.s[p.i] < '0' || p.s[p.i] > '9') return false;
    while (p.i < p.n && p.s[p.i] >= '0' && p.s[p.i] <= '9') ++p.i;
  }
  if (p.i < p.n && (p.s[p.i] == 'e' || p.s[p.i] == 'E')) {
    plain = false;
    ++p.i;
    if (p.i < p.n && (p.s[p.i] == '+' || p.s[p.i] == '-')) ++p.i;
    if (p.i >= p.n || p.s[p.i] < '0' || p.s[p.i] > '9') return false;
    while (p.i < p.n && p.s[p.i] >= '0' && p.s[p.i] <= '9') ++p.i;
  }
  std::string txt(p.s + b, p.i - b);
  v = std::strtod(txt.c_str(), nullptr);
  integral_exact = false;
  if (plain && txt.size() <= 19) {
    iv = std::strtoll(txt.c_str(), nullptr, 10);
    integral_exact = true;
  }
  return true;
}

// ---- generic value -> canonical JSON.stringify text ----
bool canonValue(Parser& p, std::string& o);

bool isArrayIndex(const std::u16string& k, uint64_t& idx) {
  if (k.empty() || k.size() > 10) return false;
  if (k.size() > 1 && k[0] == u'0') return false;
  uint64_t v = 0;
  for (char16_t c : k) {
    if (c < u'0' || c > u'9') return false;
    v = v * 10 + (c - u'0');
  }
  if (v >= 4294967295ULL) return false;
  idx = v;
  return true;
}

bool canonObject(Parser& p, std::string& o) {
  std::vector<std::pair<std::u16string, std::string>> props;
  if (p.eat('}')) {
    o += "{}";
    return true;
  }
  for (;;) {
    std::u16string key;
    if (!parseString(p, key)) return false;
    if (!p.eat(':')) return false;
    std::string val;
    if (!canonValue(p, val)) return false;
    bool dup = false;
    for (auto& kv : props)
      if (kv.first == key) { kv.second = std::move(val); dup = true; break; }
    if (!dup) props.emplace_back(std::move(key), std::move(val));
    if (p.eat(',')) continue;
    if (p.eat('}')) break;
    return false;
  }
  // JS own-property order: array indices ascending, then strings in insertion order
  std::vector<std::pair<uint64_t, size_t>> idx;
  std::vector<size_t> rest;
  for (size_t k = 0; k < props.size(); ++k) {
    uint64_t v;
    if (isArrayIndex(props[k].first, v)) idx.emplace_back(v, k);
    else rest.push_back(k);
  }
  std::sort(idx.begin(), idx.end());
  o.push_back('{');
  bool first = true;
  auto emit = [&](size_t k) {
    if (!first) o.push_back(',');
    first = false;
    quote(o, props[k].first);
    o.push_back(':');
    o += props[k].second;
  };
  for (auto& x : idx) emit(x.second);
  for (size_t k : rest) emit(k);
  o.push_back('}');
  return true;
}

bool canonValue(Parser& p, std::string& o) {
  p.ws();
  if (p.i >= p.n) return false;
  if (++p.depth > 4096) return false;
  const char c = p.s[p.i];
  bool ok = true;
  if (c == '{') {
    ++p.i;
    ok = canonObject(p, o);
  } else if (c == '[') {
    ++p.i;
    o.push_back('[');
    if (!p.eat(']')) {
      for (bool first = true;; first = false) {
        if (!first) o.push_back(',');
        if (!canonValue(p, o)) { ok = false; break; }
        if (p.eat(',')) continue;
        if (p.eat(']')) break;
        ok = false;
        break;
      }
    }
    if (ok) o.push_back(']');
  } else if (c == '"') {
    std::u16string u;
    ok = parseString(p, u);
    if (ok) quote(o, u);
  } else if (c == 't' && p.n - p.i >= 4 && std::memcmp(p.s + p.i, "true", 4) == 0) {
    p.i += 4;
    o += "true";
  } else if (c == 'f' && p.n - p.i >= 5 && std::memcmp(p.s + p.i, "false", 5) == 0) {
    p.i += 5;
    o += "false";
  } else if (c == 'n' && p.n - p.i >= 4 && std::memcmp(p.s + p.i, "null", 4) == 0) {
    p.i += 4;
    o += "null";
  } else {
    double v;
    bool ie;
    long long iv;
    ok = parseNumber(p, v, ie, iv);
    if (ok) jsNumber(o, v);
  }
  --p.depth;
  return ok;
}

// ---- operation decoder ----
struct Span {
  size_t b, e;
};

// Parse an object into (key, value span) pairs, last duplicate wins.
bool objectFields(Parser& p, std::vector<std::pair<std::u16string, Span>>& f) {
  f.clear();
  if (!p.eat('{')) return false;
  if (p.eat('}')) return true;
  for (;;) {
    std::u16string key;
    if (!parseString(p, key)) return false;
    if (!p.eat(':')) return false;
    p.ws();
    const size_t b = p.i;
    std::string sink;
    if (!canonValue(p, sink)) return false;  // validates and skips
    bool dup = false;
    for (auto& kv : f)
      if (kv.first == key) { kv.second = Span{b, p.i}; dup = true; break; }
    if (!dup) f.emplace_back(std::move(key), Span{b, p.i});
    if (p.eat(',')) continue;
    if (p.eat('}')) return true;
    return false;
  }
}

const Span* field(const std::vector<std::pair<std::u16string, Span>>& f, const char16_t* name) {
  for (auto& kv : f)
    if (kv.first == name) return &kv.second;
  return nullptr;
}

// Json.Decode.int: any finite number without a fractional part.
bool decodeInt(const char* s, const Span& sp, long long& out) {
  Parser q{s, sp.e};
  q.i = sp.b;
  double v;
  bool ie;
  long long iv;
  if (!parseNumber(q, v, ie, iv)) return false;
  q.ws();
  if (q.i != sp.e) return false;
  // (beyond 2^53 the reference's platform holds the nearest double, which
  // strtod gives: JSON.parse("9007199254740993") is 9007199254740992)
  if (ie && iv <= (1LL << 53) && iv >= -(1LL << 53)) { out = iv; return true; }
  if (!std::isfinite(v) || std::floor(v) != v || std::fabs(v) >= 9.2e18) return false;
  out = static_cast<long long>(v);
  return true;
}

bool decodeIntList(const char* s, const Span& sp, std::vector<int64_t>& out) {
  Parser q{s, sp.e};
  q.i = sp.b;
  out.clear();
  if (!q.eat('[')) return false;
  if (q.eat(']')) return true;
  for (;;) {
    q.ws();
    const size_t b = q.i;
    std::string sink;
    if (!canonValue(q, sink)) return false;
    long long v;
    if (!decodeInt(s, Span{b, q.i}, v)) return false;
    out.push_back(v);
    if (q.eat(',')) continue;
    if (q.eat(']')) return true;
    return false;
  }
}

struct Out {
  std::vector<uint8_t> kind;
  std::vector<int64_t> ts;
  std::vector<uint32_t> off{0};
  std::vector<int64_t> path;
  std::vector<uint32_t> val;
  std::string vbytes;
  std::vector<uint64_t> voff{0};
};

// decoder / decoderHelp (src/CRDTree/Operation.elm:135-159), flattening Batches.
bool decodeOp(const char* s, const Span& sp, Out& out, int depth, bool* top_batch) {
  if (depth > 4096) return false;
  Parser p{s, sp.e};
  p.i = sp.b;
  std::vector<std::pair<std::u16string, Span>> f;
  if (!objectFields(p, f)) return false;
  const Span* op = field(f, u"op");
  if (!op) return false;
  Parser q{s, op->e};
  q.i = op->b;
  std::u16string kind;
  if (!parseString(q, kind)) return false;  // field "op" Decode.string
  if (kind == u"add") {
    if (top_batch) *top_batch = false;
    const Span* ts = field(f, u"ts");
    const Span* path = field(f, u"path");
    const Span* val = field(f, u"val");
    long long t;
    std::vector<int64_t> pv;
    if (!ts || !path || !val || !decodeInt(s, *ts, t) || !decodeIntList(s, *path, pv)) return false;
    Parser vp{s, val->e};
    vp.i = val->b;
    std::string vtxt;
    if (!canonValue(vp, vtxt)) return false;
    out.kind.push_back(CRDTM_ADD);
    out.ts.push_back(t);
    out.path.insert(out.path.end(), pv.begin(), pv.end());
    out.off.push_back(static_cast<uint32_t>(out.path.size()));
    out.val.push_back(static_cast<uint32_t>(out.voff.size() - 1));
    out.vbytes += vtxt;
    out.voff.push_back(out.vbytes.size());
    return true;
  }
  if (kind == u"del") {
    if (top_batch) *top_batch = false;
    const Span* path = field(f, u"path");
    std::vector<int64_t> pv;
    if (!path || !decodeIntList(s, *path, pv)) return false;
    out.kind.push_back(CRDTM_DELETE);
    out.ts.push_back(0);
    out.path.insert(out.path.end(), pv.begin(), pv.end());
    out.off.push_back(static_cast<uint32_t>(out.path.size()));
    out.val.push_back(0);
    return true;
  }
  if (top_batch) *top_batch = true;
  if (kind != u"batch") return true;  // unknown op -> Batch []
  const Span* ops = field(f, u"ops");
  if (!ops) return false;
  Parser a{s, ops->e};
  a.i = ops->b;
  if (!a.eat('[')) return false;
  if (a.eat(']')) return true;
  for (;;) {
    a.ws();
    const size_t b = a.i;
    std::string sink;
    if (!canonValue(a, sink)) return false;
    if (!decodeOp(s, Span{b, a.i}, out, depth + 1, nullptr)) return false;
    if (a.eat(',')) continue;
    if (a.eat(']')) return true;
    return false;
  }
}

template <class T>
T* dup(const std::vector<T>& v) {
  T* p = static_cast<T*>(std::malloc(v.size() * sizeof(T) + 8));
  if (p && !v.empty()) std::memcpy(p, v.data(), v.size() * sizeof(T));
  return p;
}

// (beyond 2^53 as JSON.stringify prints the double: shortest digits, zero
// padded — a decoded value there is already a double's exact integer)
void encodeInt(std::string& o, int64_t v) {
  if (v <= (1LL << 53) && v >= -(1LL << 53)) o += std::to_string(v);
  else jsNumber(o, static_cast<double>(v));
}

void encodeOp(std::string& o, const crdtm_ops* ops, uint64_t i, const char* vb, const uint64_t* voff) {
  const uint32_t b = ops->path_off[i], e = ops->path_off[i + 1];
  if (ops->kind[i] == CRDTM_ADD) {
    o += "{\"op\":\"add\",\"path\":[";
    for (uint32_t j = b; j < e; ++j) {
      if (j > b) o.push_back(',');
      encodeInt(o, ops->path[j]);
    }
    o += "],\"ts\":";
    encodeInt(o, ops->ts[i]);
    o += ",\"val\":";
    const uint32_t h = ops->val[i];
    o.append(vb + voff[h], voff[h + 1] - voff[h]);
    o.push_back('}');
  } else {
    o += "{\"op\":\"del\",\"path\":[";
    for (uint32_t j = b; j < e; ++j) {
      if (j > b) o.push_back(',');
      encodeInt(o, ops->path[j]);
    }
    o += "]}";
  }
}

}  // namespace

extern "C" int crdtm_json_decode(const char* json, size_t len, crdtm_ops** ops, char** val_bytes, uint64_t** val_off,
                                 uint64_t* n_vals, int* is_batch) {
  if (!json || !ops) return CRDTM_E_ARG;
  Out out;
  bool top = false;
  Parser p{json, len};
  p.ws();
  const size_t b = p.i;
  std::string sink;
  if (!canonValue(p, sink)) return CRDTM_E_PARSE;
  const size_t e = p.i;
  p.ws();
  if (p.i != len) return CRDTM_E_PARSE;
  if (!decodeOp(json, Span{b, e}, out, 0, &top)) return CRDTM_E_PARSE;
  auto* r = static_cast<crdtm_ops*>(std::calloc(1, sizeof(crdtm_ops)));
  r->n_ops = out.kind.size();
  r->n_path = out.path.size();
  r->kind = dup(out.kind);
  r->ts = dup(out.ts);
  r->path_off = dup(out.off);
  r->path = dup(out.path);
  r->val = dup(out.val);
  r->tree = nullptr;
  *ops = r;
  if (val_bytes) {
    *val_bytes = static_cast<char*>(std::malloc(out.vbytes.size() + 1));
    std::memcpy(*val_bytes, out.vbytes.data(), out.vbytes.size());
    (*val_bytes)[out.vbytes.size()] = 0;
  }
  if (val_off) *val_off = dup(out.voff);
  if (n_vals) *n_vals = out.voff.size() - 1;
  if (is_batch) *is_batch = top ? 1 : 0;
  return CRDTM_OK;
}

extern "C" int crdtm_json_encode(const crdtm_ops* ops, int is_batch, const char* val_bytes, const uint64_t* val_off,
                                 char** out, size_t* out_len) {
  if (!ops || !out) return CRDTM_E_ARG;
  if (!is_batch && ops->n_ops != 1) return CRDTM_E_ARG;
  std::string o;
  o.reserve(ops->n_ops * 48 + 32);
  if (is_batch) {
    o += "{\"op\":\"batch\",\"ops\":[";
    for (uint64_t i = 0; i < ops->n_ops; ++i) {
      if (i) o.push_back(',');
      encodeOp(o, ops, i, val_bytes, val_off);
    }
    o += "]}";
  } else {
    encodeOp(o, ops, 0, val_bytes, val_off);
  }
  char* r = static_cast<char*>(std::malloc(o.size() + 1));
  std::memcpy(r, o.data(), o.size());
  r[o.size()] = 0;
  *out = r;
  if (out_len) *out_len = o.size();
  return CRDTM_OK;
}

// JSON.stringify(JSON.parse(text)) for one value (Decode.value / Encode.value).
extern "C" int crdtm_json_canonical(const char* text, size_t len, char** out, size_t* out_len) {
  if (!text || !out) return CRDTM_E_ARG;
  Parser p{text, len};
  std::string o;
  if (!canonValue(p, o)) return CRDTM_E_PARSE;
  p.ws();
  if (p.i != len) return CRDTM_E_PARSE;
  char* r = static_cast<char*>(std::malloc(o.size() + 1));
  std::memcpy(r, o.data(), o.size());
  r[o.size()] = 0;
  *out = r;
  if (out_len) *out_len = o.size();
  return CRDTM_OK;
}
