// Host-only decoding of an encoded agg param (poc/mastic.py:413-435,
// Mastic.encode_agg_param) and the evaluated prefix tree of
// eval_with_siblings (poc/vidpf.py:213-261).  Plain C++17, no HIP: the
// library builds its device tree from it (mastic_hip.hip build_tree), and the
// host sanitizer / fuzz test (tests/host/fuzz_host.cpp, built with
// -fsanitize=address,undefined) drives it with malformed and random inputs.
//
// The agg param comes from the collector, i.e. it is untrusted input: every
// malformed encoding returns TREE_EINVAL with the reference's ValueError text
// (vidpf.py:229-239, mastic.py:413-420), and a tree too large for this build
// returns TREE_ENOMEM; nothing is read outside [enc, enc + len).
#pragma once
#include <stdint.h>

#include <algorithm>
#include <cstring>
#include <new>
#include <string>
#include <vector>

enum { TREE_OK = 0, TREE_EINVAL = -22, TREE_ENOMEM = -12 };

// Node paths are at most 8 words (256 bits) in the level kernels
// (kernels.hpp node_proof_one, AesArgs child paths): BITS <= 256 covers
// every BASELINE config (C3 is BITS = 256).
constexpr int TREE_MAX_BITS = 256;
// Nodes of one tree (the host arrays hold 40 B per node, the device ones 44 B)
constexpr uint64_t TREE_MAX_NODES = 1ull << 28;

struct TreeShape {
    int L = 0;
    int n_prefixes = 0;
    bool weight_check = false;
    std::vector<int> n_parents;        // per level
    std::vector<int> n_exp;            // expanded nodes per level
    std::vector<size_t> off;           // per-level offset into the node arrays
    std::vector<int32_t> child_exp;    // per node: index in the next level's frontier, -1 = not expanded
    std::vector<int32_t> child_pfx;    // per node of level L: index in the prefix list, -1 = none
    std::vector<uint32_t> child_path;  // 8 words per node: MSB-first path bits, bytes little-endian in words
    std::vector<size_t> poff;          // per-level offset into parent_node
    std::vector<int32_t> parent_node;  // node index (in level l-1) of every parent of level l
    uint64_t nodes = 0, interior = 0;
    int max_level_nodes = 0, max_exp = 0, max_parents = 0;
};

inline int tree_fail(std::string* err, int code, const char* msg) {
    if (err) *err = msg;
    return code;
}

// Decode enc (len bytes) for a VIDPF of `bits` bits and build the tree into
// *t.  Level l's nodes are both children of every expanded node of level
// l-1, in lexicographic order, which is exactly the BFS order of the binders
// (mastic.py:263-275; the order depends only on the prefix SET).
inline int tree_parse(int bits, const uint8_t* enc, size_t len, TreeShape* t, std::string* err) {
    try {
        if (!enc || len < 7) return tree_fail(err, TREE_EINVAL, "agg param too short");
        const int level = (enc[0] << 8) | enc[1];
        const uint64_t count = ((uint64_t)enc[2] << 24) | ((uint64_t)enc[3] << 16) | ((uint64_t)enc[4] << 8) | enc[5];
        const size_t plen = (size_t)(level + 1 + 7) / 8;
        // len != 6 + plen * count + 1, without overflow (plen <= 8192, count < 2^32)
        if ((len - 7) % plen != 0 || (len - 7) / plen != count)
            return tree_fail(err, TREE_EINVAL, "agg param has incorrect length");
        if (level >= bits) return tree_fail(err, TREE_EINVAL, "level too deep");
        if (enc[len - 1] > 1) return tree_fail(err, TREE_EINVAL, "invalid weight check flag");
        // the poc cannot evaluate an empty candidate set either (eval_with_siblings leaves the
        // root's children unset and prep_init fails at mastic.py:270)
        if (count == 0) return tree_fail(err, TREE_EINVAL, "empty candidate prefix list");
        if (count > (uint64_t)INT32_MAX / 2) return tree_fail(err, TREE_EINVAL, "number of prefixes out of range");
        if (bits > TREE_MAX_BITS) return tree_fail(err, TREE_EINVAL, "BITS above 256 is not supported");
        const uint8_t* pre = enc + 6;
        const int n = (int)count;
        auto P = [&](int i) { return pre + plen * (size_t)i; };
        // bits past level + 1 must be zero (PrefixTreeIndex.encode of a length-(level+1) prefix)
        const int tail_bits = (level + 1) % 8;
        if (tail_bits) {
            const uint8_t mask = (uint8_t)((1u << (8 - tail_bits)) - 1);
            for (int i = 0; i < n; i++)
                if (P(i)[plen - 1] & mask) return tree_fail(err, TREE_EINVAL, "prefix with incorrect length");
        }
        // Sorted candidate order (lexicographic = MSB-first bit order) and the
        // common-prefix length in bits of each adjacent pair: the distinct
        // length-m prefixes are the runs of sorted candidates split wherever
        // the adjacent common prefix is shorter than m, so every level's
        // expanded nodes, child indices and paths come from O(count) scans.
        std::vector<int> order(n);
        for (int i = 0; i < n; i++) order[i] = i;
        std::sort(order.begin(), order.end(), [&](int a, int b) { return std::memcmp(P(a), P(b), plen) < 0; });
        auto bit_of = [&](int s, int l) { return (P(order[s])[l / 8] >> (7 - l % 8)) & 1; };
        std::vector<int> lcp(n, -1);  // lcp[0] = -1: always starts a run
        for (int s = 1; s < n; s++) {
            const uint8_t* a = P(order[s - 1]);
            const uint8_t* b = P(order[s]);
            size_t k = 0;
            while (k < plen && a[k] == b[k]) k++;
            if (k == plen) return tree_fail(err, TREE_EINVAL, "candidate prefixes are non-unique");
            lcp[s] = (int)k * 8 + __builtin_clz((unsigned)(a[k] ^ b[k])) - 24;
        }
        // nodes before any allocation: level l has 2 x (runs at length l) nodes,
        // runs at length l = 1 + #{s : lcp[s] < l}
        uint64_t all_nodes = 0;
        {
            std::vector<uint64_t> below(level + 2, 0);  // below[m] = #{s >= 1 : lcp[s] < m}
            for (int s = 1; s < n; s++) below[std::min(lcp[s] + 1, level + 1)]++;
            uint64_t runs = 0;
            for (int l = 0; l <= level; l++) {
                runs += below[l];
                all_nodes += 2 * (1 + runs);
                if (all_nodes > TREE_MAX_NODES) return tree_fail(err, TREE_ENOMEM, "agg param tree too large");
            }
        }
        TreeShape& T = *t;
        T = TreeShape();
        T.child_exp.resize(all_nodes);
        T.child_pfx.resize(all_nodes);
        T.child_path.resize(8 * all_nodes);
        T.parent_node.reserve(all_nodes / 2);
        T.L = level;
        T.n_prefixes = n;
        T.weight_check = enc[len - 1] == 1;
        size_t total = 0;
        std::vector<int> run_begin;        // runs of length-l prefixes = parents of level l
        std::vector<int> gid_next(n, 0);   // run index of each sorted candidate at length l+1
        run_begin.push_back(0);            // level 0: the root (one run over all candidates)
        for (int l = 0; l <= level; l++) {
            const int np = (int)run_begin.size();
            T.n_parents.push_back(np);
            T.poff.push_back(T.parent_node.size());
            if (l > 0) {
                // parents of level l are level l-1's expanded nodes; their node index
                const size_t prev = T.off[l - 1];
                const int prev_nodes = 2 * T.n_parents[l - 1];
                for (int k = 0; k < prev_nodes; k++)
                    if (T.child_exp[prev + k] >= 0) T.parent_node.push_back(k);
            }
            int n_next = 0;
            std::vector<int> next_begin;
            if (l < level) {
                for (int s = 0; s < n; s++) {
                    if (lcp[s] < l + 1) {
                        next_begin.push_back(s);
                        n_next++;
                    }
                    gid_next[s] = n_next - 1;
                }
            }
            T.n_exp.push_back(n_next);
            T.off.push_back(total);
            for (int pi = 0; pi < np; pi++) {
                const int b = run_begin[pi];
                const int e = pi + 1 < np ? run_begin[pi + 1] : n;
                const uint8_t* rep = P(order[b]);
                // the parent's path: the run's first l bits (MSB-first bytes,
                // bits past l zero); word k holds bytes 4k..4k+3 little-endian
                uint8_t pb[32] = {0};
                std::memcpy(pb, rep, (size_t)(l / 8));
                if (l % 8) pb[l / 8] = (uint8_t)(rep[l / 8] & (0xFF00u >> (l % 8)));
                for (int cbit = 0; cbit < 2; cbit++) {
                    // child cbit exists iff the run's first (cbit 0) / last (cbit 1)
                    // member has that bit at position l
                    const int m = cbit ? e - 1 : b;
                    const bool exists = bit_of(m, l) == cbit;
                    int ce = -1, cp = -1;
                    if (exists) {
                        if (l < level)
                            ce = gid_next[m];
                        else
                            cp = order[m];
                    }
                    const size_t node = total + 2 * (size_t)pi + cbit;
                    T.child_exp[node] = ce;
                    T.child_pfx[node] = cp;
                    // path: the parent's l bits, then cbit (bits past l + 1 zero)
                    if (cbit) pb[l / 8] |= (uint8_t)(0x80u >> (l % 8));
                    uint32_t* w = T.child_path.data() + 8 * node;
                    for (int k = 0; k < 8; k++)
                        w[k] = (uint32_t)pb[4 * k] | (uint32_t)pb[4 * k + 1] << 8 | (uint32_t)pb[4 * k + 2] << 16 |
                               (uint32_t)pb[4 * k + 3] << 24;
                }
            }
            total += 2 * (size_t)np;
            T.max_level_nodes = std::max(T.max_level_nodes, 2 * np);
            T.max_parents = std::max(T.max_parents, np);
            T.max_exp = std::max(T.max_exp, T.n_exp.back());
            if (l > 0) T.interior += np;
            run_begin.swap(next_begin);
        }
        T.nodes = total;
        return TREE_OK;
    } catch (const std::bad_alloc&) {
        return tree_fail(err, TREE_ENOMEM, "out of host memory (agg param tree)");
    }
}
