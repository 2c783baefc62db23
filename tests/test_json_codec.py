"""Wire format (src/CRDTree/Operation.elm:109-159), CPU only.

tests/JsonTest.elm:20-62 pins encode->decode round trips; the byte format
itself is pinned by tests/golden/json_values.json, generated from node's own
JSON.stringify/JSON.parse (tests/golden/make_json_fixtures.js) — the platform
`Json.Encode.encode 0` runs on.
"""
import json
import os

import pytest

from crdtm.codec import DecodeError, canonical_value, decoder, encoder
from crdtm.operation import Add, Batch, Delete

GOLD = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "json_values.json")))


# tests/JsonTest.elm:20-62
@pytest.mark.parametrize("op", [Add(3, [1, 2], "a"), Delete([1, 2]),
                                Batch([Add(3, [1, 2], "a"), Add(4, [1, 3], "b"), Delete([1, 2])])])
def test_round_trip(op):
    assert decoder(encoder(op)) == op


@pytest.mark.parametrize("case", GOLD["values"], ids=lambda c: c["input"][:24])
def test_value_canonical_matches_node(case):
    assert canonical_value(case["input"]) == case["output"]


def test_op_bytes_match_node():
    ops = [Add(3, [1, 2], "a"), Delete([1, 2]),
           Batch([Add(3, [1, 2], "a"), Add(4, [1, 3], "b"), Delete([1, 2])]),
           Add(4294967297, [0], {"k": [1, 2.5, "x"]}), Batch([])]
    for op, want in zip(ops, GOLD["ops"]):
        assert encoder(op) == want
        assert decoder(want) == op


def test_decoder_semantics():
    # unknown "op" -> Batch [] (src/CRDTree/Operation.elm:158-159), also nested
    assert decoder('{"op":"nope"}') == Batch([])
    assert decoder('{"op":"batch","ops":[{"op":"x"},{"op":"del","path":[5]}]}') == Batch([Delete([5])])
    # nested batches flatten in order
    assert decoder('{"op":"batch","ops":[{"op":"batch","ops":[{"op":"del","path":[1]}]},{"op":"del","path":[2]}]}') \
        == Batch([Delete([1]), Delete([2])])
    # Decode.int accepts integral numbers in any form, rejects fractions
    assert decoder('{"op":"add","ts":1e2,"path":[2.0],"val":null}') == Add(100, [2], None)
    with pytest.raises(DecodeError):
        decoder('{"op":"add","ts":1.5,"path":[0],"val":1}')
    # field order does not matter; extra fields are ignored; missing fields fail
    assert decoder(' {"val":"v","x":1,"path":[0],"op":"add","ts":7} ') == Add(7, [0], "v")
    for bad in ('{"op":"add","path":[0],"val":1}', '{"op":"del"}', '{"path":[1]}', '{"op":5}', '[]', '{"op":"add"',
                '{"op":"batch"}'):
        with pytest.raises(DecodeError):
            decoder(bad)
