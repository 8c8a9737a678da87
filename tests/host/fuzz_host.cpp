// Host sanitizer + fuzz driver for the untrusted-input decoders of the
// library: the agg-param decoder / tree builder
// (csrc/host_tree.hpp, used by mastic_hip.hip build_tree) and the parameter
// derivation (csrc/params.hpp mc_derive, used by mastic_ctx_create).
// Built by tests/test_host_sanitize.py with
//   g++ -std=c++17 -O1 -g -fsanitize=address,undefined -fno-sanitize-recover=all
// and run on the CPU; any sanitizer report aborts the run.
//
// Checks:
//  * every malformed encoding the reference rejects returns TREE_EINVAL with
//    the reference's ValueError text (poc/vidpf.py:229-239, poc/mastic.py:413-420);
//  * valid encodings build exactly the tree of a naive restatement of
//    Vidpf.eval_with_siblings' node set (poc/vidpf.py:240-261), BFS order;
//  * random mutations of valid encodings (bit flips, truncation, extension,
//    header rewrites) never crash and return only OK / EINVAL / ENOMEM, with
//    a consistent tree when OK;
//  * mc_derive over random and extreme parameters: no UB, sizes positive.
// Prints one line per named case and "fuzz_host: OK" at the end.
#include <cstdio>
#include <cstdlib>
#include <map>
#include <random>
#include <set>
#include <string>
#include <vector>

#include "../../draft-mouris-cfrg-mastic_amd/csrc/host_tree.hpp"
#include "../../draft-mouris-cfrg-mastic_amd/csrc/params.hpp"

typedef std::vector<bool> Path;

static int failures = 0;
#define CHECK(cond, ...)                                              \
    do {                                                              \
        if (!(cond)) {                                                \
            fprintf(stderr, "FAIL %s:%d: ", __FILE__, __LINE__);      \
            fprintf(stderr, __VA_ARGS__);                             \
            fprintf(stderr, "\n");                                    \
            if (++failures > 20) exit(1);                             \
        }                                                             \
    } while (0)

// Mastic.encode_agg_param (poc/mastic.py:413-435)
static std::vector<uint8_t> encode(int level, const std::vector<Path>& prefixes, int wc) {
    std::vector<uint8_t> e = {(uint8_t)(level >> 8), (uint8_t)level};
    const uint32_t n = (uint32_t)prefixes.size();
    for (int s = 24; s >= 0; s -= 8) e.push_back((uint8_t)(n >> s));
    const size_t plen = (size_t)(level + 1 + 7) / 8;
    for (const Path& p : prefixes) {
        std::vector<uint8_t> b(plen, 0);
        for (size_t i = 0; i < p.size(); i++)
            if (p[i]) b[i / 8] |= (uint8_t)(0x80 >> (i % 8));
        e.insert(e.end(), b.begin(), b.end());
    }
    e.push_back((uint8_t)wc);
    return e;
}

static std::vector<uint32_t> path_words(const Path& p) {
    std::vector<uint32_t> w(8, 0);
    for (size_t i = 0; i < p.size(); i++)
        if (p[i]) w[i / 32] |= 0x80u >> (i % 8) << (8 * ((i / 8) % 4));
    return w;
}

// Naive restatement of the evaluated node set of eval_with_siblings
// (vidpf.py:240-261): level l holds both children of every distinct
// length-l prefix of a candidate; a node is expanded (evaluated further) iff
// it is a length-(l+1) prefix of a candidate below level L.
static void check_against_naive(const TreeShape& T, int level, const std::vector<Path>& pfx) {
    size_t off = 0;
    for (int l = 0; l <= level; l++) {
        std::set<Path> parents;
        for (const Path& p : pfx) parents.insert(Path(p.begin(), p.begin() + l));
        std::vector<Path> nodes;
        for (const Path& q : parents)
            for (int b = 0; b < 2; b++) {
                Path c = q;
                c.push_back(b != 0);
                nodes.push_back(c);
            }
        CHECK((int)parents.size() == T.n_parents[l], "level %d parents %zu vs %d", l, parents.size(), T.n_parents[l]);
        CHECK(T.off[l] == off, "level %d offset", l);
        std::set<Path> exp;
        if (l < level)
            for (const Path& p : pfx) exp.insert(Path(p.begin(), p.begin() + l + 1));
        std::map<Path, int> exp_idx;
        for (const Path& e : exp) exp_idx.emplace(e, (int)exp_idx.size());
        CHECK((int)exp.size() == T.n_exp[l], "level %d expanded", l);
        for (size_t k = 0; k < nodes.size() && off + k < T.child_exp.size(); k++) {
            const Path& c = nodes[k];
            auto it = exp_idx.find(c);
            CHECK(T.child_exp[off + k] == (it == exp_idx.end() ? -1 : it->second), "level %d node %zu exp", l, k);
            int want_pfx = -1;
            if (l == level)
                for (size_t i = 0; i < pfx.size(); i++)
                    if (pfx[i] == c) want_pfx = (int)i;
            CHECK(T.child_pfx[off + k] == want_pfx, "level %d node %zu pfx", l, k);
            const std::vector<uint32_t> w = path_words(c);
            for (int j = 0; j < 8; j++) CHECK(T.child_path[(off + k) * 8 + j] == w[j], "level %d node %zu path", l, k);
        }
        off += nodes.size();
    }
    CHECK(T.nodes == off, "nodes");
}

static void check_consistent(const TreeShape& T) {
    uint64_t total = 0;
    for (size_t l = 0; l < T.n_parents.size(); l++) {
        CHECK(T.off[l] == total, "offsets");
        const int nn = 2 * T.n_parents[l];
        for (int k = 0; k < nn; k++) {
            const int ce = T.child_exp[total + k];
            CHECK(ce >= -1 && ce < T.n_exp[l], "child_exp range");
            const int cp = T.child_pfx[total + k];
            CHECK(cp >= -1 && cp < T.n_prefixes, "child_pfx range");
        }
        if (l + 1 < T.n_parents.size()) CHECK(T.n_exp[l] == T.n_parents[l + 1], "frontier -> parents");
        total += nn;
    }
    CHECK(T.nodes == total && T.child_path.size() == 8 * total, "sizes");
}

static void expect(const char* name, int bits, const std::vector<uint8_t>& e, int want_rc, const char* want_msg) {
    TreeShape T;
    std::string err;
    const int rc = tree_parse(bits, e.data(), e.size(), &T, &err);
    printf("case %-28s rc=%d err=%s\n", name, rc, err.c_str());
    CHECK(rc == want_rc, "%s: rc %d, want %d", name, rc, want_rc);
    if (want_msg) CHECK(err == want_msg, "%s: '%s', want '%s'", name, err.c_str(), want_msg);
}

static Path rand_path(std::mt19937_64& g, int n) {
    Path p(n);
    for (int i = 0; i < n; i++) p[i] = (g() & 1) != 0;
    return p;
}

static std::vector<Path> rand_prefixes(std::mt19937_64& g, int level, int count) {
    std::set<Path> s;
    const int want = level < 20 ? std::min(count, 1 << (level + 1)) : count;
    // clustered: share random leading bits so runs and siblings occur
    const Path base = rand_path(g, level + 1);
    while ((int)s.size() < want) {
        Path p = base;
        const int keep = (int)(g() % (level + 2));
        for (int i = keep; i <= level; i++) p[i] = (g() & 1) != 0;
        s.insert(p);
    }
    return std::vector<Path>(s.begin(), s.end());
}

int main() {
    std::mt19937_64 g(0x4D41);
    // ---- named malformed inputs (reference ValueError text) ----
    {
        const std::vector<Path> two = {Path{false, true, false, true, true, false}, Path{true, true, false, false, true, true}};
        const std::vector<uint8_t> ok = encode(5, two, 1);
        expect("valid", 8, ok, TREE_OK, nullptr);
        expect("empty", 8, {}, TREE_EINVAL, "agg param too short");
        expect("six bytes", 8, std::vector<uint8_t>(ok.begin(), ok.begin() + 6), TREE_EINVAL, "agg param too short");
        expect("truncated body", 8, std::vector<uint8_t>(ok.begin(), ok.end() - 2), TREE_EINVAL,
               "agg param has incorrect length");
        std::vector<uint8_t> longer = ok;
        longer.insert(longer.end() - 1, 0);
        expect("oversized body", 8, longer, TREE_EINVAL, "agg param has incorrect length");
        std::vector<uint8_t> hugecount = ok;
        hugecount[2] = 0x80;  // count = 2^31 + 2 with a two-prefix body
        expect("count >= 2^31", 8, hugecount, TREE_EINVAL, "agg param has incorrect length");
        hugecount[2] = 0xff, hugecount[3] = hugecount[4] = hugecount[5] = 0xff;
        expect("count = 2^32 - 1", 8, hugecount, TREE_EINVAL, "agg param has incorrect length");
        expect("level == bits", 5, ok, TREE_EINVAL, "level too deep");
        std::vector<uint8_t> flag = ok;
        flag.back() = 2;
        expect("weight check flag 2", 8, flag, TREE_EINVAL, "invalid weight check flag");
        expect("zero prefixes", 8, encode(5, {}, 0), TREE_EINVAL, "empty candidate prefix list");
        std::vector<uint8_t> tail = ok;
        tail[6] |= 0x01;  // bit 7 set on a 6-bit prefix
        expect("non-zero tail bits", 8, tail, TREE_EINVAL, "prefix with incorrect length");
        expect("duplicate prefixes", 8, encode(5, {two[0], two[1], two[0]}, 0), TREE_EINVAL,
               "candidate prefixes are non-unique");
        expect("BITS 257", 257, ok, TREE_EINVAL, "BITS above 256 is not supported");
        std::vector<uint8_t> maxlevel = ok;
        maxlevel[0] = maxlevel[1] = 0xff;  // level 65535: length check first
        expect("level 65535", 256, maxlevel, TREE_EINVAL, "agg param has incorrect length");
        // a valid encoding whose tree exceeds TREE_MAX_NODES: 2^20 prefixes at level 255
        // (random 256-bit prefixes: distinct with overwhelming probability)
        std::vector<uint8_t> big = {0, 255, 0x00, 0x10, 0x00, 0x00};
        for (size_t i = 0; i < (32u << 20); i++) big.push_back((uint8_t)g());
        big.push_back(0);
        expect("tree too large", 256, big, TREE_ENOMEM, "agg param tree too large");
    }
    // ---- valid encodings against the naive node set ----
    int checked = 0;
    const int bits_choices[] = {1, 2, 3, 5, 8, 9, 16, 31, 32, 64, 200, 256};
    for (int it = 0; it < 1500; it++) {
        const int bits = bits_choices[g() % (sizeof bits_choices / sizeof bits_choices[0])];
        const int level = (int)(g() % bits);
        const int count = 1 + (int)(g() % 24);
        std::vector<Path> pfx = rand_prefixes(g, level, count);
        std::shuffle(pfx.begin(), pfx.end(), g);
        TreeShape T;
        std::string err;
        const std::vector<uint8_t> e = encode(level, pfx, (int)(g() & 1));
        const int rc = tree_parse(bits, e.data(), e.size(), &T, &err);
        CHECK(rc == TREE_OK, "valid encoding rejected: %s", err.c_str());
        if (rc == TREE_OK) {
            check_against_naive(T, level, pfx);
            check_consistent(T);
            checked++;
        }
    }
    printf("case %-28s %d trees equal to the naive node set\n", "naive", checked);
    // ---- mutation fuzz ----
    int n_ok = 0, n_inval = 0, n_nomem = 0;
    for (int it = 0; it < 60000; it++) {
        const int bits = bits_choices[g() % (sizeof bits_choices / sizeof bits_choices[0])];
        const int level = (int)(g() % bits);
        std::vector<uint8_t> e = encode(level, rand_prefixes(g, level, 1 + (int)(g() % 6)), (int)(g() % 2));
        const int kind = (int)(g() % 6);
        const int nm = 1 + (int)(g() % 3);
        for (int k = 0; k < nm; k++) {
            if (kind == 0 && !e.empty()) e[g() % e.size()] ^= (uint8_t)(1u << (g() % 8));
            if (kind == 1 && !e.empty()) e.resize(g() % e.size());
            if (kind == 2) e.push_back((uint8_t)g());
            if (kind == 3 && e.size() > 6) e[2 + g() % 4] = (uint8_t)g();  // count
            if (kind == 4 && e.size() > 2) e[g() % 2] = (uint8_t)g();      // level
            if (kind == 5 && !e.empty()) e[g() % e.size()] = (uint8_t)g();
        }
        TreeShape T;
        std::string err;
        // the buffer is exactly e.size() bytes: ASan flags any read past it
        std::vector<uint8_t> exact(e);
        const int rc = tree_parse(bits, exact.empty() ? nullptr : exact.data(), exact.size(), &T, &err);
        CHECK(rc == TREE_OK || rc == TREE_EINVAL || rc == TREE_ENOMEM, "rc %d", rc);
        if (rc == TREE_OK) {
            n_ok++;
            check_consistent(T);
        } else if (rc == TREE_EINVAL) {
            n_inval++;
            CHECK(!err.empty(), "EINVAL without text");
        } else {
            n_nomem++;
        }
    }
    printf("case %-28s ok=%d einval=%d enomem=%d\n", "mutations", n_ok, n_inval, n_nomem);
    // ---- mc_derive ----
    int derived = 0;
    const int64_t extremes[] = {-2147483647 - 1, -1, 0, 1, 2, 63, 64, 255, 256, 257, 1024, 65535, 65536,
                                (1 << 22), (1 << 22) + 1, 2147483647};
    for (int it = 0; it < 100000; it++) {
        auto pick = [&]() -> int {
            if (g() % 3 == 0) return (int)extremes[g() % (sizeof extremes / sizeof extremes[0])];
            return (int)(g() % 5000) - 10;
        };
        const int circuit = (int)(g() % 7);
        uint64_t maxm = g() % 4 == 0 ? g() : g() % 300;
        McParams p;
        if (mc_derive(circuit, pick(), pick(), (int)(g() % 70) - 3, maxm, pick(), &p) == 0) {
            derived++;
            CHECK(p.value_len >= 2 && p.proof_len > 0 && p.verifier_len > 0, "derived sizes");
            CHECK(mc_public_share_size(p) > 0 && mc_input_share_size(p, 0) > 0 && mc_input_share_size(p, 1) > 0,
                  "wire sizes");
        }
    }
    printf("case %-28s %d valid of 100000\n", "mc_derive", derived);
    if (failures) {
        printf("fuzz_host: %d FAILURES\n", failures);
        return 1;
    }
    printf("fuzz_host: OK\n");
    return 0;
}
