// Generates tests/golden/json_values.json: inputs and JSON.stringify(JSON.parse(x))
// outputs from node's own JSON implementation (the platform Elm's
// Json.Encode.encode 0 / Json.Decode run on; SURVEY.md A.10). Run:
//   node tests/golden/make_json_fixtures.js > tests/golden/json_values.json
const inputs = [
  '"a"', '"\\u00e9t\\u00e9"', '"tab\\there"', '"nl\\n"', '"quote\\"q"', '"back\\\\slash"', '"slash\\/x"',
  '"ctl\\u0001\\u001f"', '"del\\u007f"', '"\\ud83d\\ude00"', '"lone\\ud800x"', '"lone\\udfff"', '"\\uD83D\\uDE00"',
  '"raw é ü 中"', '"😀"', '"\\b\\f\\r"', '""',
  '0', '-0', '1', '-1', '1.0', '1.5', '-2.25', '1e2', '1E2', '1e21', '1e20', '123456789012345678901', '1e-6',
  '1e-7', '0.000001', '0.0000001', '1.5e-7', '3.14159', '2e308', '-1e-400', '0.1', '0.30000000000000004',
  '9007199254740993', '4294967296', '12345678.9', '1.23e+5', '5e-324', '1.7976931348623157e308',
  'true', 'false', 'null', '[]', '{}', '[1,"a",null]', ' [ 1 , 2 ] ',
  '{"b":1,"a":2}', '{"a":1,"a":2}', '{"2":"x","1":"y","b":"z","10":"w","01":"v"}', '{"a":{"c":[1,{"d":2}],"b":0}}',
  '{"4294967294":1,"4294967295":2,"x":3}', '{"-1":1,"0":2}', '{"a":1,"b":2,"a":3}',
];
const out = inputs.map((s) => ({ input: s, output: JSON.stringify(JSON.parse(s)) }));
const ops = [
  { op: 'add', path: [1, 2], ts: 3, val: 'a' },
  { op: 'del', path: [1, 2] },
  { op: 'batch', ops: [{ op: 'add', path: [1, 2], ts: 3, val: 'a' }, { op: 'add', path: [1, 3], ts: 4, val: 'b' }, { op: 'del', path: [1, 2] }] },
  { op: 'add', path: [0], ts: 4294967297, val: { k: [1, 2.5, 'x'] } },
  { op: 'batch', ops: [] },
];
console.log(JSON.stringify({ generator: 'node ' + process.version, values: out,
  ops: ops.map((o) => JSON.stringify(o)) }, null, 1));
