"""CPU restatement of Corda's partial Merkle trees (test infrastructure: the
checker for the GPU path, never the product path).

Follows, line by line in behaviour:
  PartialMerkleTree.build          core/.../crypto/PartialMerkleTree.kt:68-78
  checkFull                        PartialMerkleTree.kt:80-91
  buildPartialTree                 PartialMerkleTree.kt:100-125
  PartialMerkleTree.verify         PartialMerkleTree.kt:132-158
  FilteredTransaction.verify       core/.../transactions/MerkleTransaction.kt:134-140
  MerkleTree.getMerkleTree         core/.../crypto/MerkleTree.kt:27-66 (padWithZeros, zeroHash = 32 x 0x00)
  SecureHash.hashConcat            core/.../crypto/SecureHash.kt:24 (SHA-256(left || right))

Trees are nested tuples: ("leaf", h) / ("node", h, left, right) for MerkleTree,
("incl", h) / ("leaf", h) / ("node", left, right) for PartialTree.

The device-side encoding (include/cordahip.h, cordahip_filtered_tx_verify) is
the post-order token stream of a PartialTree: 0 = IncludedLeaf(hash),
1 = Leaf(hash), 2 = Node (pops right, then left).
"""
import hashlib

ZERO = bytes(32)
TOK_INCL, TOK_LEAF, TOK_NODE = 0, 1, 2


class MerkleTreeException(Exception):
    pass


def hash_concat(a: bytes, b: bytes) -> bytes:
    return hashlib.sha256(a + b).digest()


def merkle_tree(leaf_hashes):
    """MerkleTree.getMerkleTree (MerkleTree.kt:27-66)."""
    if not leaf_hashes:
        raise MerkleTreeException("Cannot calculate Merkle root on empty hash list.")
    n = 1
    while n < len(leaf_hashes):
        n *= 2
    level = [("leaf", h) for h in leaf_hashes] + [("leaf", ZERO)] * (n - len(leaf_hashes))
    while len(level) > 1:
        level = [("node", hash_concat(level[i][1], level[i + 1][1]), level[i], level[i + 1])
                 for i in range(0, len(level), 2)]
    return level[0]


def _check_full(tree, level=0):
    if tree[0] == "leaf":
        return level
    l1 = _check_full(tree[2], level + 1)
    l2 = _check_full(tree[3], level + 1)
    if l1 != l2:
        raise MerkleTreeException("Got not full binary tree.")
    return l1


def _build_partial(root, include, used):
    if root[0] == "leaf":
        if root[1] in include:
            used.append(root[1])
            return True, ("incl", root[1])
        return False, ("leaf", root[1])
    lf, lt = _build_partial(root[2], include, used)
    rf, rt = _build_partial(root[3], include, used)
    if lf or rf:
        return True, ("node", lt, rt)
    return False, ("leaf", root[1])


def build(merkle_root, include_hashes):
    """PartialMerkleTree.build (PartialMerkleTree.kt:68-78)."""
    if ZERO in include_hashes:
        raise ValueError("Zero hashes shouldn't be included in partial tree.")
    _check_full(merkle_root)
    used = []
    _, tree = _build_partial(merkle_root, include_hashes, used)
    if len(include_hashes) != len(used):
        raise MerkleTreeException("Some of the provided hashes are not in the tree.")
    return tree


def _verify_rec(node, used):
    if node[0] == "incl":
        used.append(node[1])
        return node[1]
    if node[0] == "leaf":
        return node[1]
    return hash_concat(_verify_rec(node[1], used), _verify_rec(node[2], used))


def verify(partial_tree, merkle_root_hash, hashes_to_check):
    """PartialMerkleTree.verify (PartialMerkleTree.kt:132-139): multiset of the
    included hashes == multiset of hashes_to_check, and the recomputed root."""
    used = []
    root = _verify_rec(partial_tree, used)
    if sorted(hashes_to_check) != sorted(used):  # groupBy { it } equality == multiset equality
        return False
    return root == merkle_root_hash


def filtered_tx_verify(root_hash, filtered_leaf_hashes, partial_tree):
    """FilteredTransaction.verify (MerkleTransaction.kt:134-140)."""
    if not filtered_leaf_hashes:
        raise MerkleTreeException("Transaction without included leaves.")
    return verify(partial_tree, root_hash, filtered_leaf_hashes)


def tokens(partial_tree):
    """Post-order token stream: [(tok, hash_or_None), ...]."""
    out = []

    def rec(n):
        if n[0] == "incl":
            out.append((TOK_INCL, n[1]))
        elif n[0] == "leaf":
            out.append((TOK_LEAF, n[1]))
        else:
            rec(n[1])
            rec(n[2])
            out.append((TOK_NODE, None))

    rec(partial_tree)
    return out


def verify_tokens(toks, root_hash, hashes_to_check):
    """The stack-machine reading of verify() the GPU kernel implements; None = malformed stream."""
    stack, used = [], []
    for t, h in toks:
        if t == TOK_INCL:
            used.append(h)
            stack.append(h)
        elif t == TOK_LEAF:
            stack.append(h)
        elif t == TOK_NODE:
            if len(stack) < 2:
                return None
            r = stack.pop()
            left = stack.pop()
            stack.append(hash_concat(left, r))
        else:
            return None
    if len(stack) != 1:
        return None
    if sorted(hashes_to_check) != sorted(used):
        return False
    return stack[0] == root_hash
