"""Known-answer scenarios shared by the oracle KATs and the GPU parity tests.

Transcribed from the reference's own tests (tests/CRDTreeTest.elm,
tests/NodeTest.elm — file:line per case) and from the hand-traced vectors of
SURVEY.md Appendix C. Each scenario is a replica id plus a sequence of
top-level `apply` calls (an Add/Delete or a Batch), so the same case drives
the oracle and the HIP engine.
"""
from crdtm.operation import Add, Batch, Delete

T32 = 2 ** 32

# name -> (replica, [top-level ops applied in turn])
SCENARIOS = {
    # tests/CRDTreeTest.elm:125-160 (addAfter2: [a, z, b, c])
    "add_after2": (0, [Batch([Add(1, [0], "a"), Add(2, [1], "b"), Add(3, [2], "c"), Add(4, [1], "z")])]),
    # tests/CRDTreeTest.elm:202-258 (nested branches)
    "add_branch": (0, [Batch([Add(1, [0], "a"), Add(2, [1, 0], "b"), Add(3, [1, 2, 0], "c"),
                              Add(4, [1, 2, 3, 0], "d"), Add(5, [1, 2, 3, 4, 0], "e"),
                              Add(6, [1, 2, 3, 4, 5], "f")])]),
    # tests/CRDTreeTest.elm:261-278
    "delete": (0, [Add(1, [0], "a"), Delete([1])]),
    # tests/CRDTreeTest.elm:281-321 (add under a deleted branch: dropped, not logged)
    "add_to_deleted_branch": (0, [Batch([Add(1, [0], "a"), Delete([1]), Add(2, [1, 0], "b")])]),
    # tests/CRDTreeTest.elm:324-358
    "apply_batch": (0, [Batch([Add(1, [0], "a"), Add(2, [1], "b")])]),
    # tests/CRDTreeTest.elm:361-398
    "add_idempotent": (0, [Batch([Add(1, [0], "a")] * 4)]),
    # tests/CRDTreeTest.elm:401-440
    "insertion_between": (0, [Batch([Add(1, [0], "a"), Add(2, [1], "c"), Add(3, [1], "b")])]),
    # tests/CRDTreeTest.elm:443-479
    "add_leaf": (0, [Batch([Add(1, [0], "a"), Add(2, [1, 0], "b"), Add(3, [1, 2], "c")])]),
    # tests/CRDTreeTest.elm:482-498 (atomicity: Add 2 [9] fails the batch)
    "atomicity": (0, [Batch([Add(1, [0], "a"), Add(2, [9], "b")])]),
    # tests/CRDTreeTest.elm:501-544
    "delete_idempotent": (0, [Batch([Add(1, [0], "a")] + [Delete([1])] * 5)]),
    # tests/CRDTreeTest.elm:547-589 (replica 1 offsets)
    "timestamps_r1": (1, [Batch([Add(T32 + 1, [0], "a"), Add(T32 + 2, [T32 + 1], "b"),
                                 Add(T32 + 3, [T32 + 2], "c")])]),
    # tests/CRDTreeTest.elm:592-658
    "operations_since": (0, [Batch([Add(1, [0], "a"), Add(2, [1], "b"), Add(3, [2], "c"), Add(4, [3], "d"),
                                    Delete([3]), Batch([]), Add(5, [4], "e"), Add(6, [5], "f")])]),
    # tests/NodeTest.elm:138-147 (append both orders -> [b, a])
    "append_smaller_first": (0, [Add(1, [0], "a"), Add(2, [0], "b")]),
    "append_bigger_first": (0, [Add(2, [0], "b"), Add(1, [0], "a")]),
    # tests/NodeTest.elm:150-167 (-> [1,6,5,4,2,3])
    "insert_smaller_first": (0, [Add(1, [0], 1), Add(2, [1], 2), Add(3, [2], 3), Add(6, [1], 6), Add(5, [1], 5),
                                 Add(4, [1], 4)]),
    "insert_bigger_first": (0, [Add(1, [0], 1), Add(2, [1], 2), Add(3, [2], 3), Add(4, [1], 4), Add(6, [1], 6),
                                Add(5, [1], 5)]),
    # tests/NodeTest.elm:170-177 (flat with tombstone x)
    "flat_example": (0, [Add(1, [0], "a"), Add(2, [1], "b"), Add(3, [2], "x"), Add(4, [3], "c"), Add(5, [4], "d"),
                         Delete([3])]),
    # tests/NodeTest.elm:180-185
    "nested_example": (0, [Add(1, [0], "a"), Add(2, [1, 0], "b"), Add(3, [1, 2, 0], "c"),
                           Add(4, [1, 2, 3, 0], "d")]),
    # the copy quirk (findInsertion skips tombstone 20)
    "quirk_copy": (0, [Batch([Add(10, [0], "p"), Add(20, [10], "q"), Add(30, [20], "r"), Delete([20]),
                              Add(15, [10], "s")]), Delete([30])]),
    # Appendix C.2: same adds, deletes last (order-dependence witness)
    "quirk_deletes_last": (0, [Batch([Add(10, [0], "p"), Add(20, [10], "q"), Add(30, [20], "r"),
                                      Add(15, [10], "s"), Delete([20]), Delete([30])])]),
    # Appendix C.3: non-Lamport order -> visible [1,5,3,2]
    "non_lamport": (0, [Batch([Add(1, [0], 1), Add(5, [1], 5), Add(2, [5], 2), Add(3, [1], 3)])]),
    # Appendix C.4: Delete [0] on a fresh tree -> Ok, nothing logged
    "delete_sentinel": (0, [Delete([0])]),
    # Appendix C.5: Add under the sentinel -> ignored
    "add_under_sentinel": (0, [Add(7, [0, 0], "x")]),
    # Appendix C.6: AlreadyApplied still bumps the own timestamp; Delete records the deleted ts
    "replica_accounting": (1, [Batch([Add(T32 + 1, [0], "a"), Add(T32 + 1, [0], "a"),
                                      Add(2 * T32 + 1, [T32 + 1], "b"), Delete([2 * T32 + 1])])]),
    # Error paths (src/CRDTree.elm:321-325): InvalidPath / OperationFailed
    "invalid_path_empty": (0, [Batch([Add(1, [0], "a"), Delete([])])]),
    "invalid_path_missing_parent": (0, [Batch([Add(1, [0], "a"), Add(2, [5, 0], "b")])]),
    "delete_missing": (0, [Batch([Add(1, [0], "a"), Delete([7])])]),
    # Quirk copying a branch with children (persistent copy of the subtree)
    "quirk_copy_branch": (0, [Batch([Add(10, [0], "p"), Add(20, [10], "q"), Add(30, [20], "r"),
                                     Add(31, [30, 0], "r1"), Delete([20]), Add(15, [10], "s"),
                                     Add(32, [20, 31], "via-copy"), Add(33, [30, 31], "via-orphan")])]),
    # Trailing tombstones stop the walk (Appendix A.5)
    "trailing_tombstones": (0, [Batch([Add(10, [0], "p"), Add(30, [10], "q"), Add(40, [30], "r"),
                                       Delete([30]), Delete([40]), Add(20, [10], "s")])]),
    # Anchor is a tombstone
    "anchor_tombstone": (0, [Batch([Add(10, [0], "p"), Add(20, [10], "q"), Delete([20]), Add(25, [20], "s"),
                                    Add(5, [20], "t")])]),
    # Negative and zero timestamps
    "odd_timestamps": (0, [Batch([Add(-5, [0], "n"), Add(0, [0], "z"), Add(3, [-5], "p"), Add(-9, [0], "m")])]),
    # Two remote replicas concurrently typing after the same anchor
    "two_replicas": (0, [Batch([Add(T32 + 1, [0], "a"), Add(2 * T32 + 1, [0], "b"), Add(T32 + 2, [T32 + 1], "c"),
                                Add(2 * T32 + 2, [2 * T32 + 1], "d"), Add(T32 + 3, [2 * T32 + 2], "e")])]),
    # Incremental applies onto an existing tree
    "incremental": (0, [Batch([Add(1, [0], "a"), Add(2, [1], "b")]), Batch([Add(3, [1], "c"), Delete([2])]),
                        Batch([Add(4, [3], "d"), Add(5, [0], "e")])]),
}
