// Integers past 2^53 through the reference's platform (node: JSON.parse then
// JSON.stringify in the encoder's key order, src/CRDTree/Operation.elm:109-159):
//   node tests/golden/make_bigint_fixtures.js > tests/golden/json_bigint.json
const xs = ["9007199254740991", "9007199254740992", "9007199254740993", "-9007199254740993",
            "9007199254740995", "1234567890123456789", "-1234567890123456789", "4611686018427387904",
            "9.007199254740993e15", "1e18"];
const cases = [];
for (const x of xs) {
  const t = "{\"op\":\"add\",\"ts\":" + x + ",\"path\":[" + x + ",0],\"val\":1}";
  const o = JSON.parse(t);
  cases.push({input: t, output: JSON.stringify({op: "add", path: o.path, ts: o.ts, val: o.val})});
}
process.stdout.write(JSON.stringify({node: process.version, cases: cases}, null, 1) + "\n");
