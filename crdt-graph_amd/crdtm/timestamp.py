"""CRDTree.Timestamp mirror (src/CRDTree/Timestamp.elm:16-18).

replicaId ts = ts // 2^32, where Elm's `//` on JS numbers is (a / b) | 0:
truncation toward zero (exact for |ts| < 2^53).
"""

TWO32 = 2 ** 32


def replica_id(ts: int) -> int:
    q = abs(int(ts)) // TWO32
    return q if ts >= 0 else -q
