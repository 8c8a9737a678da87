"""VIDPF-proof aggregation mode.

draft-mouris-cfrg-mastic.md, "Plain Heavy-Hitters with VIDPF-Proof
Aggregation": the two aggregators compute identical eval proofs for a report
iff it is valid (mastic.py:340 compares them per report), so instead of
exchanging every prep share they compare a Merkle tree over the batch's eval
proofs and interactively descend into the subtrees whose hashes differ to
isolate the invalid reports.  Best case (all valid): one 32-byte root per
batch; worst case O(n) hashes over log2(n) rounds.

The draft gives no hash, tree shape or wire format (it is a TODO there) and
the poc has no code for it, so this module fixes them (parity unpinned
against the reference; the GPU tree is checked against a CPU construction
in tests/test_gpu_proof_agg.py):
  * leaves = the n eval proofs in report order;
  * parent of (left, right) = XofTurboShake128(b'', dst(ctx, 12), left || right).next(32)
    with dst(ctx, usage) = b'mastic' || 0x00 || usage || ctx (poc/dst.py:30-32,
    usage 12 is new);
  * the last node of an odd level is promoted unchanged.
The GPU builds the tree (``Mastic.proof_tree``, C ABI ``mastic_proof_tree``).
"""


def level_sizes(n: int):
    """Node counts per level, leaves first: n, ceil(n/2), ..., 1 (none for n = 0)."""
    sizes = []
    m = n
    while m > 0:
        sizes.append(m)
        m = 0 if m == 1 else (m + 1) // 2
    return sizes


def isolate_invalid(tree_a, tree_b):
    """Interactive traversal between the two aggregators' trees (lists of
    levels, leaves first).  Starting at the roots, the children of every node
    pair that differs are compared next.  Returns (indices of the leaves whose
    eval proofs differ, number of node hashes one aggregator sent, rounds)."""
    if len(tree_a) != len(tree_b) or any(len(x) != len(y) for (x, y) in zip(tree_a, tree_b)):
        raise ValueError("proof trees have different shapes")
    if not tree_a:
        return ([], 0, 0)
    top = len(tree_a) - 1
    frontier = [0] if tree_a[top][0] != tree_b[top][0] else []
    sent, rounds = 1, 1
    for lv in range(top, 0, -1):
        if not frontier:
            break
        below = len(tree_a[lv - 1])
        nxt = []
        for i in frontier:
            for c in (2 * i, 2 * i + 1):
                if c < below:
                    sent += 1
                    if tree_a[lv - 1][c] != tree_b[lv - 1][c]:
                        nxt.append(c)
        frontier = nxt
        rounds += 1
    return (frontier, sent, rounds)
