// Generates tests/golden/json_ops.json: operation JSON texts in deliberately
// non-canonical forms (random key order, whitespace, numbers written with
// exponents or trailing zeros, escaped characters) and, for each, the bytes
// `Json.Encode.encode 0 (encoder Encode.value op)` produces for the decoded
// operation: JSON.stringify of the op object in the encoder's key order
// (src/CRDTree/Operation.elm:109-129) — node's own JSON implementation, the
// platform elm/json runs on (SURVEY.md A.10). Batches are one level deep
// (the host decoder flattens nested Batches, which `apply` treats alike).
// Run:  node tests/golden/make_op_fixtures.js > tests/golden/json_ops.json
let s = 0x5eed1234;
const rnd = () => { s ^= s << 13; s >>>= 0; s ^= s >>> 17; s ^= s << 5; s >>>= 0; return s / 4294967296; };
const pick = (a) => a[Math.floor(rnd() * a.length)];
const chars = ['a', 'b', 'Z', ' ', '"', '\\', '/', '\n', '\t', '\r', '\b', '\f', '\u0001', '\u001f', '\u007f', 'é',
  '中', '😀', '\ud800', '\udfff', '0', '{', '}', '[', ']', ',', ':'];
function rstring() { let t = ''; const n = Math.floor(rnd() * 8); for (let i = 0; i < n; ++i) t += pick(chars); return t; }
function rnumber() {
  return pick([0, -0, 1, -1, 7, 255, 4294967296, 9007199254740991, -9007199254740991, 0.5, -2.25, 3.14159, 1e21,
    1e-7, 123456.789, 5e-324, 1.7976931348623157e308, Math.floor(rnd() * 1e6) / 8]);
}
function rvalue(d) {
  const k = Math.floor(rnd() * (d > 2 ? 4 : 6));
  if (k === 0) return rstring();
  if (k === 1) return rnumber();
  if (k === 2) return pick([true, false, null]);
  if (k === 3) return rstring() + rstring();
  if (k === 4) { const a = []; const n = Math.floor(rnd() * 4); for (let i = 0; i < n; ++i) a.push(rvalue(d + 1)); return a; }
  const o = {}; const n = Math.floor(rnd() * 4);
  for (let i = 0; i < n; ++i) o[pick(['a', 'b', 'k', '2', '10', '01', '-1', 'x y', 'é', '4294967295'])] = rvalue(d + 1);
  return o;
}
const ws = () => pick(['', '', ' ', '\n', '\t ', '  ']);
// a number in some valid JSON spelling that JSON.parse maps to x
function numText(x) {
  if (Object.is(x, -0)) return pick(['-0', '-0.0', '-0e0']);
  if (Number.isInteger(x) && Math.abs(x) < 1e15 && x !== 0 && rnd() < 0.3) {
    const m = pick(['e0', '.0', '.000', 'E0']);
    return String(x) + m;
  }
  if (Number.isInteger(x) && x % 100 === 0 && x !== 0 && Math.abs(x) < 1e15 && rnd() < 0.5) return String(x / 100) + 'e2';
  return JSON.stringify(x);
}
function strText(t) {  // JSON string with some characters escaped in alternative ways
  let o = '"';
  for (const c of t) {
    const code = c.codePointAt(0);
    if (c === '"') o += '\\"';
    else if (c === '\\') o += '\\\\';
    else if (c === '/' && rnd() < 0.5) o += '\\/';
    else if (code < 0x20 || (code >= 0xd800 && code <= 0xdfff) || (code < 0x10000 && rnd() < 0.2))
      o += '\\u' + code.toString(16).padStart(4, '0');  // (a lone surrogate is never raw: the input is UTF-8)
    else if (code >= 0x10000 && rnd() < 0.5) {
      const h = c.charCodeAt(0), l = c.charCodeAt(1);
      o += '\\u' + h.toString(16) + '\\u' + l.toString(16).toUpperCase();
    } else o += c;
  }
  return o + '"';
}
function text(v) {  // a non-canonical serialisation of a JSON value
  if (v === null || typeof v === 'boolean') return String(v);
  if (typeof v === 'number') return numText(v);
  if (typeof v === 'string') return strText(v);
  if (Array.isArray(v)) return '[' + ws() + v.map((e) => text(e)).join(ws() + ',' + ws()) + ws() + ']';
  const keys = Object.keys(v);
  for (let i = keys.length - 1; i > 0; --i) { const j = Math.floor(rnd() * (i + 1)); [keys[i], keys[j]] = [keys[j], keys[i]]; }
  return '{' + ws() + keys.map((k) => strText(k) + ws() + ':' + ws() + text(v[k])).join(',' + ws()) + ws() + '}';
}
function objText(fields) {  // an op object with its fields in random order
  const ks = Object.keys(fields);
  for (let i = ks.length - 1; i > 0; --i) { const j = Math.floor(rnd() * (i + 1)); [ks[i], ks[j]] = [ks[j], ks[i]]; }
  return '{' + ws() + ks.map((k) => '"' + k + '"' + ws() + ':' + ws() + fields[k]).join(',' + ws()) + ws() + '}';
}
const rint = () => pick([0, 1, 3, 4294967297, 9007199254740991, Math.floor(rnd() * 2 ** 40)]);
function leaf() {
  const path = []; const L = 1 + Math.floor(rnd() * 4);
  for (let i = 0; i < L; ++i) path.push(rint());
  const ptext = '[' + path.map((p) => numText(p)).join(',' + ws()) + ']';
  if (rnd() < 0.7) {
    const ts = rint(), vtext = text(rvalue(0));
    // Decode.value then Encode.value: the value as JSON.parse reads the text
    // (object keys in text order, array-index keys first)
    return { canon: { op: 'add', path, ts, val: JSON.parse(vtext) },
      text: objText({ op: '"add"', path: ptext, ts: numText(ts), val: vtext, extra: text(rvalue(1)) }) };
  }
  return { canon: { op: 'del', path }, text: objText({ op: '"del"', path: ptext }) };
}
const cases = [];
for (let k = 0; k < 300; ++k) {
  if (rnd() < 0.25) {
    const n = Math.floor(rnd() * 5), ls = [];
    for (let i = 0; i < n; ++i) ls.push(leaf());
    const parts = ls.map((l) => l.text);
    if (rnd() < 0.3) parts.push('{"op":"unknown","x":1}');  // unknown op inside: Batch [] (flattens to nothing)
    cases.push({ input: objText({ op: '"batch"', ops: '[' + parts.join(',' + ws()) + ']' }),
      output: JSON.stringify({ op: 'batch', ops: ls.map((l) => l.canon) }) });
  } else {
    const l = leaf();
    cases.push({ input: l.text, output: JSON.stringify(l.canon) });
  }
}
console.log(JSON.stringify({ generator: 'node ' + process.version, seed: '0x5eed1234', cases }, null, 1));
