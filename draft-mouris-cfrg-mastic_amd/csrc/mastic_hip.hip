// Host side of the MI355X Mastic aggregator: C ABI (include/mastic_hip.h),
// agg-param decoding and tree building, HBM buffer management and the
// level-by-level launch schedule.  No CPU compute path exists: every
// cryptographic operation of prep_init / shard / decide / aggregate runs in
// the kernels of kernels.hpp / shard.hpp.
#include "mastic_hip.h"

#include <dlfcn.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <system_error>
#include <thread>
#include <type_traits>
#include <vector>

#include "comm_agree.hpp"
#include "host_tree.hpp"
#include "kernels.hpp"
#include "shard.hpp"

namespace {

// MASTIC_TRACE_ALLOC=1: log every device allocation / free with its duration (stderr)
static bool trace_alloc() {
    static const bool on = [] {
        const char* e = getenv("MASTIC_TRACE_ALLOC");
        return e && e[0] == '1';
    }();
    return on;
}
// MASTIC_TRACE_COMM=1: log the communicator's init / agreement / abort steps (stderr)
static bool trace_comm() {
    static const bool on = [] {
        const char* e = getenv("MASTIC_TRACE_COMM");
        return e && e[0] == '1';
    }();
    return on;
}
static double now_ms() {
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

struct DevBuf {
    void* p = nullptr;
    size_t bytes = 0;
    bool own = true;  // false: a view into another buffer (mastic_reports_view)
    ~DevBuf() { release(); }
    void release() {
        if (p && own) {
            const double t0 = trace_alloc() ? now_ms() : 0;
            (void)hipFree(p);
            if (trace_alloc()) fprintf(stderr, "[mastic] free %.3f GB %.1f ms\n", bytes / 1e9, now_ms() - t0);
        }
        p = nullptr;
        bytes = 0;
        own = true;
    }
    void view(const DevBuf& b, size_t off, size_t len) {
        release();
        if (!b.p) return;
        p = (uint8_t*)b.p + off;
        bytes = len;
        own = false;
    }
    bool ensure(size_t want) {
        if (want <= bytes && p) return true;
        release();
        if (want == 0) want = 16;
        const double t0 = trace_alloc() ? now_ms() : 0;
        const hipError_t e = hipMalloc(&p, want);
        if (trace_alloc()) fprintf(stderr, "[mastic] malloc %.3f GB %.1f ms%s\n", want / 1e9, now_ms() - t0,
                                   e == hipSuccess ? "" : " FAILED");
        if (e != hipSuccess) {
            p = nullptr;
            (void)hipGetLastError();  // callers handle it; keep it out of later launch checks
            return false;
        }
        bytes = want;
        return true;
    }
    // ensure() with headroom: buffers that follow a growing size (results,
    // staging) are re-allocated rarely (a large hipMalloc costs ~1 s per
    // 50 GB on MI355X)
    bool grow(size_t want) {
        if (want <= bytes && p) return true;
        return ensure(std::max(want, bytes + bytes / 2)) || ensure(want);
    }
    template <class T> T* as() const { return (T*)p; }
};

// The decoded agg param's tree (host_tree.hpp) plus its device copy.
// The device arrays live in one allocation (dev): child_exp, child_pfx,
// child_path, parent_node.
struct Tree : TreeShape {
    DevBuf dev;
    int32_t* d_exp = nullptr;
    int32_t* d_pfx = nullptr;
    uint32_t* d_path = nullptr;
    int32_t* d_parent = nullptr;
};

struct Result {
    bool ready = false;
    size_t n = 0, stride = 0;
    int weight_check = 0;
    int n_prefixes = 0;
    DevBuf out, eval_proof, verifier, jr_part, jr_seed, status;
};

inline size_t round_up(size_t x, size_t m) { return (x + m - 1) / m * m; }

// Frontier cache of one aggregator (mastic_set_frontier_cache; SURVEY.md §8f
// row 1).  In a level sweep (examples.py:37-91) prep_init at level L evaluates
// the whole tree again, but its levels 0..L-1 are usually exactly the previous
// call's tree.  The cache keeps, per report, the two binder sponges' states
// after the cached call's levels (the binder messages are BFS-ordered, so the
// cached message is a prefix of the next one), every node of the last level as
// its convert seed and control bit (5 words: a hit recomputes a parent's seed
// and payload from its convert stream), and the root sum; a call whose tree
// extends the cached one by one level evaluates and absorbs only that level.
// Planes of all n reports (stride S, independent of the HBM-budget chunks a
// call runs in, so a sweep's chunking may change from level to level).  The
// last level kernel writes its children straight into a spare node slot
// shared by the ctx's aggregators (mastic_ctx::fc_spare; a hit reads its
// parents from this aggregator's slot meanwhile), and the call then swaps the
// two: three node slots in all, no copy of the level into the cache.
struct LevelCache {
    bool valid = false;
    uint64_t rep_id = 0, rep_gen = 0;  // the batch (mastic_reports::id) and its contents generation
    size_t n = 0;
    size_t S = 0;                               // plane stride (n rounded up to 64, plus padding)
    std::vector<uint8_t> key;                   // u8(len) || verify key || ctx
    int L = -1;                                 // level of the cached call
    std::vector<int> n_parents;                 // per level 0..L
    std::vector<uint32_t> paths;                // child paths of level L (8 words per node)
    DevBuf sp, rootsum;                         // both binder sponges (2 x 50 planes); root sum (wl planes)
    DevBuf nd;                                  // last level's nodes [node][5]: convert seed, control bit
    size_t nodes_cap = 0;                       // nodes nd can hold
    void drop() { valid = false; }
    void release() {
        drop();
        sp.release();
        rootsum.release();
        nd.release();
        nodes_cap = 0;
        S = 0;
    }
};

}  // namespace

// Frontier-cache key of a batch: its identity (id, unique per batch or view
// object) and the generation of the HBM it reads.  A batch and its views share
// one generation counter (`gen`), so an upload or shard through any of them
// invalidates cache entries keyed on the others.  Contexts may be driven from
// several threads, so the counters are atomic.
static std::atomic<uint64_t> g_reports_gen{0};
static uint64_t next_reports_gen() { return g_reports_gen.fetch_add(1) + 1; }
struct mastic_reports {
    mastic_ctx* ctx = nullptr;
    size_t n = 0;
    uint64_t id = next_reports_gen();
    std::shared_ptr<std::atomic<uint64_t>> gen = std::make_shared<std::atomic<uint64_t>>(next_reports_gen());
    DevBuf nonces, pub, in0, in1;
    void touch() { gen->store(next_reports_gen()); }
    uint64_t generation() const { return gen->load(); }
};

struct mastic_ctx {
    mastic_params user{};
    McParams p{};
    int device = 0;
    hipStream_t stream = nullptr;   // level evals, setup, finalize, FLP
    hipStream_t stream2 = nullptr;  // binder sponges (overlap the next level's eval)
    hipStream_t stream3 = nullptr;  // binder sponges of the odd chunks of a pipelined prep_init
    hipStream_t stream4 = nullptr;  // FLP randomness + query of a weight-check call, beside its last sponges
    std::vector<hipEvent_t> sync_ev;
    hipEvent_t fold_ev = nullptr;  // mastic_fold_shares: producer stream -> stream
    hipEvent_t comm_marks[3] = {};  // MASTIC_TRACE_COMM: progress marks of the agreement round
    // library-owned RCCL communicator (mastic_comm_init; none = world 1)
    ncclComm_t comm = nullptr;
    int comm_n = 1, comm_rank = 0;
    bool comm_broken = false;  // aborted after a failed / timed-out step: collective calls fail
    int comm_timeout_ms = MASTIC_COMM_TIMEOUT_MS;  // bound of every wait on the communicator
    DevBuf comm_local, comm_gather, comm_out;  // mastic_aggregate_merged / mastic_allgather_fold staging
    DevBuf comm_st;                            // agreement round: this rank's status + every rank's
    void* comm_st_host = nullptr;              // pinned host copy of the same (nranks + 1 records)
    size_t comm_st_host_n = 0;
    void comm_release();                       // teardown of a live communicator (defined with the RCCL binding)
    PrefixState pfx_host[PFX_COUNT];
    std::string err;
    uint64_t budget = 0;
    DevBuf work;     // per-chunk planes
    DevBuf pfx;      // PrefixState[PFX_COUNT]
    DevBuf pfx_bytes, pfx_meta;
    DevBuf consts;   // alpha^-i table for prove
    DevBuf agg_valid, agg_out;  // mastic_aggregate staging
    DevBuf agg_part;            // per-chunk partial sums of a split fold (aggregate_impl)
    DevBuf stage;               // result encoding / decide staging
    // Lanes per binder sponge.  Two (k_absorb_pair: half the dependent chain
    // per permutation, ~1.5x the VALU issue slots) while the chains are the
    // critical path, i.e. a chunk of few reports (C2's 16,384: one sponge wave
    // for every second SIMD); one (k_absorb: a third fewer VALU slots taken
    // from the level kernel beside it) once a chunk has enough reports for the
    // sponges to be throughput-bound (the 1M-report sweep's ~380k-report
    // chunks).  Same-box A/B (profiles/r05_v6_ab_single_lane_sponges.txt): one
    // lane is +4.5 % on the 1M sweep, -2 % on C2 and -21 % on C5 at 16,384.
    // 0 = by chunk size (>= absorb_single_min reports: one lane), 1 = always
    // one, 2 = always two (MASTIC_ABSORB_SINGLE).
    int absorb_mode = 0;
    size_t absorb_single_min = 65536;  // MASTIC_ABSORB_SINGLE_MIN
    int absorb_lds = 0;         // bytes of dynamic LDS per absorb workgroup (MASTIC_ABSORB_LDS_KB)
    int n_cus = 256;                     // compute units of the device
    int proof_waves = EVAL_PROOF_WAVES;  // proof waves per eval workgroup (MASTIC_PROOF_WAVES)
    int hit_proof_waves = 0;             // ... of a fused-proof hit launch (0 = by the work split; MASTIC_HIT_PROOF_WAVES)
    int proof_prio = 0;                  // their s_setprio (MASTIC_PROOF_PRIO)
    int aes_prio = 0;                    // s_setprio of the AES waves (MASTIC_AES_PRIO)
    int dbg_skip = 0;                    // timing experiments only (MASTIC_DBG_SKIP; results wrong): 1 no node proofs, 2 no AES, 4 no binder sponges
    int stride_pad = 64;                 // words of padding per plane row (MASTIC_STRIDE_PAD)
    size_t work_arena = (size_t)48 << 30;  // minimum size of a new work buffer (MASTIC_WORK_ARENA_GB)
    // ... with the frontier cache on (level sweeps, whose trees grow from level to level): large
    // enough that a 1M-report C2 sweep's cache misses run as one chunk (r02 v58: -4 % sweep time)
    size_t work_arena_fc = (size_t)128 << 30;
    bool binder_tiled = true;            // tiled level binder buffers (MASTIC_BINDER_TILED=0: planes)
    int absorb_threads = 256;            // threads per binder-sponge workgroup (MASTIC_ABSORB_THREADS)
    int absorb_prio = 3;                 // s_setprio of the binder sponge waves (MASTIC_ABSORB_PRIO)
    int absorb_dbg = 0;                  // timing experiments only (MASTIC_ABSORB_DBG, kernels.hpp AbsorbArgs::dbg)
    // result-preserving test hooks (mastic_set_test_hooks; nothing in the environment sets them)
    int force_slow_blk = -1;    // exact payload stream from this block on
    int fail_allocs = 0;        // this many result / cache-slot allocations fail first (ENOMEM recovery)
    int sponge_delay_us = 0;    // the next prep_init first holds the sponge stream this long (k_spin)
    int wall_khz = 100000;      // wall_clock64() rate (hipDeviceAttributeWallClockRate)
    bool timing_nowait = false; // A/B of the last_timing fix only (MASTIC_DBG_TIMING_NOWAIT, knob builds)
    bool serial_sponges = false;  // measurement: sponge launches run alone (mastic_set_serial_sponges)
    bool inject_alloc_failure() {
        if (fail_allocs <= 0) return false;
        fail_allocs--;
        return true;
    }
    // Wait for everything queued on the ctx's three streams (explicitly: the
    // recovery paths below free buffers that queued kernels on any of them may
    // still read, so they must not rely on hipFree's implicit device wait).
    bool idle() {
        return hipStreamSynchronize(stream) == hipSuccess && hipStreamSynchronize(stream2) == hipSuccess &&
               hipStreamSynchronize(stream3) == hipSuccess && hipStreamSynchronize(stream4) == hipSuccess;
    }
    int split_sponges = -1;  // payload sponge a level earlier, on the third stream: -1 Field128 only, 0 never, 1 always (MASTIC_SPLIT_SPONGES)
    bool fuse_last_miss = false;    // any miss's last level with fused, overlapped node proofs (MASTIC_FUSE_LAST_MISS=1)
    bool fuse_last_miss_fc = true;  // ... a cache-on miss's (MASTIC_FUSE_LAST_MISS_FC=0: k_node_proof)
    bool hit_absorb_main = true;  // a single-chunk hit's sponges on the main stream (MASTIC_HIT_ABSORB_MAIN=0: sponge stream)
    bool fc_all = false;        // A/B only: the frontier-cache kernel variant at every level (MASTIC_FC_ALL=1)
    bool small_split = true;    // small levels' parents split into block-range items (MASTIC_SMALL_SPLIT=0: off)
    int fuse_proofs = 1;        // last level's node proofs in the level kernel, overlapped with its AES: 1 on
                                // cache hits, 2 also on cache-on misses, 0 never (MASTIC_FUSE_PROOFS; else
                                // k_node_proof); 3 (A/B): on hits, after a workgroup barrier
    size_t chunk_max = 0;        // reports per chunk cap (0 = what fits; MASTIC_CHUNK_REPORTS)
    bool chunk_pipeline = true;  // several chunks: two halves of the work arena (MASTIC_CHUNK_PIPELINE=0: off)
    int par_waves = 0;           // waves' worth of parents per level-kernel workgroup (0 = by field; MASTIC_PAR_WAVES)
    int pfx_f[PFX_COUNT] = {0};  // fill position of each prefix state (host copy)
    std::vector<uint8_t> pfx_key;  // verify key || ctx of the prefix states in pfx (empty: none)
    std::map<std::vector<uint8_t>, Tree*> trees;
    Result res[2];
    bool frontier_cache = false;  // mastic_set_frontier_cache
    bool last_hit = false;        // the last prep_init evaluated only its last level
    LevelCache lc[2];
    DevBuf fc_spare;          // the frontier cache's spare node slot (LevelCache::nd layout)
    size_t spare_cap = 0;     // nodes it can hold
    size_t spare_S = 0;       // its plane stride
    std::vector<void*> graveyard;  // replaced cache slots, freed once the streams are idle
    // The AES key schedules in the work arena (k_setup): the reports, ctx and
    // plane geometry they were derived for, so a frontier-cache hit over the
    // same batch skips k_setup (the fixed keys depend on the nonce and ctx only,
    // not on the aggregator or level).  Cleared by anything else that writes
    // the arena's header (a chunked call, the shard's scratch).
    struct {
        bool valid = false;
        uint64_t rep_id = 0, rep_gen = 0;
        size_t n = 0;
        int stride = 0;
        const void* W = nullptr;
        std::vector<uint8_t> pfx_key;
    } rk;
    // pinned staging of the tree uploads (build_tree): one async copy per new
    // tree on the main stream; tree_ev marks when the staging may be reused
    void* tree_stage = nullptr;
    size_t tree_stage_bytes = 0;
    hipEvent_t tree_ev = nullptr;
    void bury() {
        for (void* q : graveyard) (void)hipFree(q);
        graveyard.clear();
    }
    // timing
    // timing events and results of the last prep_init of each aggregator
    // (both may be queued before either's results are fetched)
    struct Timing {
        std::vector<hipEvent_t> ev;
        double t_eval = 0, t_proof = 0, t_absorb = 0, t_total = 0;
        int n_eval = 0, n_absorb = 0;
    } tm[2];
    int tcur = 0;  // aggregator whose timing mastic_last_timing* report (last prep_init / prep_result)
    ~mastic_ctx() {
        bury();
        for (auto& kv : trees) delete kv.second;
        for (auto& x : tm)
            for (auto e : x.ev) (void)hipEventDestroy(e);
        for (auto e : sync_ev) (void)hipEventDestroy(e);
        if (fold_ev) (void)hipEventDestroy(fold_ev);
        for (hipEvent_t e : comm_marks)
            if (e) (void)hipEventDestroy(e);
        if (comm) comm_release();
        if (comm_st_host) (void)hipHostFree(comm_st_host);
        if (tree_ev) (void)hipEventDestroy(tree_ev);
        if (tree_stage) (void)hipHostFree(tree_stage);
        if (stream) (void)hipStreamDestroy(stream);
        if (stream2) (void)hipStreamDestroy(stream2);
        if (stream3) (void)hipStreamDestroy(stream3);
        if (stream4) (void)hipStreamDestroy(stream4);
    }
};

// Every entry point that touches the GPU runs with the ctx's device current
// (and restores the caller's), so contexts on different GPUs can be driven
// from one thread.
struct DeviceScope {
    int prev = -1;
    explicit DeviceScope(const mastic_ctx* c);
    ~DeviceScope() {
        if (prev >= 0) (void)hipSetDevice(prev);
    }
};
DeviceScope::DeviceScope(const mastic_ctx* c) {
    int cur = -1;
    if (c && hipGetDevice(&cur) == hipSuccess && cur != c->device && hipSetDevice(c->device) == hipSuccess) prev = cur;
}

static int fail(mastic_ctx* c, int code, const char* fmt, ...) {
    if (c) {
        char buf[512];
        va_list ap;
        va_start(ap, fmt);
        vsnprintf(buf, sizeof buf, fmt, ap);
        va_end(ap);
        c->err = buf;
    }
    return code;
}

#define HIPCHK(c, expr)                                                                  \
    do {                                                                                 \
        hipError_t _e = (expr);                                                          \
        if (_e != hipSuccess) return fail((c), MASTIC_EHIP, "%s: %s", #expr, hipGetErrorString(_e)); \
    } while (0)

// ---------------------------------------------------------------- helpers
static void put_le16(std::vector<uint8_t>& v, uint32_t x) {
    v.push_back((uint8_t)x);
    v.push_back((uint8_t)(x >> 8));
}

// dst (poc/dst.py:30-32) and dst_alg (:35-42)
static std::vector<uint8_t> dst(const uint8_t* ctx, size_t n, int usage) {
    std::vector<uint8_t> d = {'m', 'a', 's', 't', 'i', 'c', 0, (uint8_t)usage};
    d.insert(d.end(), ctx, ctx + n);
    return d;
}
static std::vector<uint8_t> dst_alg(const uint8_t* ctx, size_t n, int usage, uint32_t id) {
    std::vector<uint8_t> d = {'m', 'a', 's', 't', 'i', 'c', 0, (uint8_t)usage,
                              (uint8_t)(id >> 24), (uint8_t)(id >> 16), (uint8_t)(id >> 8), (uint8_t)id};
    d.insert(d.end(), ctx, ctx + n);
    return d;
}

// Compute the sponge prefix states for (ctx, verify_key) on the device.  The
// verify key is XofTurboShake128's seed (u8 length prefix, mastic.py:302-306,
// 499-510), so any length up to 255 bytes is accepted (the reference's own
// driver uses 16, examples.py:38,176; VERIFY_KEY_SIZE is 32, mastic.py:73).
static int build_prefixes(mastic_ctx* c, const uint8_t* app_ctx, size_t ctx_len, const uint8_t* vk, size_t vk_len) {
    if (ctx_len > 65535 - 12) return fail(c, MASTIC_EINVAL, "ctx too long");
    if (vk && vk_len > 255) return fail(c, MASTIC_EINVAL, "verify key too long");
    // callers without a verify key (decide, shard, proof tree) never read the
    // two verify-key states (PFX_EVAL, PFX_QUERY: prep_init only), so any
    // states of the same ctx serve them.  Key layout: u8(len) || vk || ctx || 1.
    if (!vk && !c->pfx_key.empty()) {
        const size_t kl = c->pfx_key[0];
        if (c->pfx_key.size() == 1 + kl + ctx_len + 1 &&
            (ctx_len == 0 || std::equal(app_ctx, app_ctx + ctx_len, c->pfx_key.begin() + 1 + kl)))
            return 0;
    }
    static const uint8_t zero_vk[32] = {0};
    if (!vk) {
        vk = zero_vk;
        vk_len = 32;
    }
    std::vector<uint8_t> key(1, (uint8_t)vk_len);
    key.insert(key.end(), vk, vk + vk_len);
    key.insert(key.end(), app_ctx, app_ctx + ctx_len);
    key.push_back(1);  // never equal to the empty "none" key
    if (key == c->pfx_key) return 0;  // same verify key and ctx as the states already in pfx
    c->pfx_key.clear();
    std::vector<std::vector<uint8_t>> m(PFX_COUNT);
    auto xof_ts = [&](int id, const std::vector<uint8_t>& d, int seed_len, const uint8_t* seed) {
        put_le16(m[id], (uint32_t)d.size());
        m[id].insert(m[id].end(), d.begin(), d.end());
        m[id].push_back((uint8_t)seed_len);
        if (seed) m[id].insert(m[id].end(), seed, seed + seed_len);
    };
    auto xof_aes = [&](int id, const std::vector<uint8_t>& d) {
        put_le16(m[id], (uint32_t)d.size());
        m[id].insert(m[id].end(), d.begin(), d.end());
    };
    const uint32_t ID = c->p.alg_id;
    xof_aes(PFX_EXT, dst(app_ctx, ctx_len, 10));
    xof_aes(PFX_CONV, dst(app_ctx, ctx_len, 11));
    xof_ts(PFX_NODE, dst(app_ctx, ctx_len, 9), 16, nullptr);
    xof_ts(PFX_ONEHOT, dst_alg(app_ctx, ctx_len, 6, ID), 0, nullptr);
    xof_ts(PFX_PAYLOAD, dst_alg(app_ctx, ctx_len, 7, ID), 0, nullptr);
    xof_ts(PFX_EVAL, dst_alg(app_ctx, ctx_len, 8, ID), (int)vk_len, vk);
    xof_ts(PFX_QUERY, dst_alg(app_ctx, ctx_len, 2, ID), (int)vk_len, vk);
    xof_ts(PFX_PROOF_SHARE, dst_alg(app_ctx, ctx_len, 1, ID), 32, nullptr);
    xof_ts(PFX_JR_PART, dst_alg(app_ctx, ctx_len, 4, ID), 32, nullptr);
    xof_ts(PFX_JR_SEED, dst_alg(app_ctx, ctx_len, 3, ID), 0, nullptr);
    xof_ts(PFX_JR, dst_alg(app_ctx, ctx_len, 5, ID), 32, nullptr);
    xof_ts(PFX_PROVE_RAND, dst_alg(app_ctx, ctx_len, 0, ID), 32, nullptr);
    xof_ts(PFX_TREE, dst(app_ctx, ctx_len, 12), 0, nullptr);
    std::vector<uint8_t> all;
    std::vector<int> meta(2 * PFX_COUNT);
    for (int i = 0; i < PFX_COUNT; i++) {
        c->pfx_f[i] = (int)(m[i].size() % KECCAK_RATE);
        meta[i] = (int)all.size();
        meta[PFX_COUNT + i] = (int)m[i].size();
        all.insert(all.end(), m[i].begin(), m[i].end());
    }
    if (!c->pfx.ensure(sizeof(PrefixState) * PFX_COUNT) || !c->pfx_bytes.ensure(all.size()) ||
        !c->pfx_meta.ensure(meta.size() * sizeof(int)))
        return fail(c, MASTIC_ENOMEM, "out of device memory (prefix states)");
    HIPCHK(c, hipMemcpyAsync(c->pfx_bytes.p, all.data(), all.size(), hipMemcpyHostToDevice, c->stream));
    HIPCHK(c, hipMemcpyAsync(c->pfx_meta.p, meta.data(), meta.size() * sizeof(int), hipMemcpyHostToDevice, c->stream));
    hipLaunchKernelGGL(k_prefix_states, dim3(1), dim3(64), 0, c->stream, c->pfx_bytes.as<uint8_t>(),
                       c->pfx_meta.as<int>(), c->pfx_meta.as<int>() + PFX_COUNT, (int)PFX_COUNT,
                       c->pfx.as<PrefixState>());
    HIPCHK(c, hipGetLastError());
    HIPCHK(c, hipMemcpyAsync(c->pfx_host, c->pfx.p, sizeof(PrefixState) * PFX_COUNT, hipMemcpyDeviceToHost,
                             c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    c->pfx_key = std::move(key);
    return 0;
}

template <class F>
static FlpConsts<F> flp_consts(const McParams& p) {
    typedef typename F::E E;
    FlpConsts<F> fc;
    // gen = 7^GEN_BASE_EXP; alpha = gen^(GEN_ORDER / P)
    const uint64_t gen_exp = p.field == 64 ? 4294967295ull : 4611686018427387897ull;
    E g = fpow_u64<F>(F::from_u64(7), gen_exp);
    int log_order = FieldConsts<F>::GEN_ORDER_LOG2;
    int logp = 0;
    while ((1 << logp) < p.P) logp++;
    int sh = log_order - logp;  // exponent 2^sh
    uint64_t ex[2] = {0, 0};
    ex[sh / 64] = 1ull << (sh % 64);
    fc.alpha = fpow<F>(g, ex, 2);
    fc.inv_p = finv<F>(F::from_u64((uint64_t)p.P));
    fc.inv2 = finv<F>(F::from_u64(2));
    fc.offset = F::from_u64(p.offset);
    fc.offset_h = F::mul(fc.offset, fc.inv2);
    return fc;
}

// ---------------------------------------------------------------- tree
// Decode Mastic.encode_agg_param (mastic.py:413-435) and build the evaluated
// prefix tree of eval_with_siblings (vidpf.py:213-261): the children of every
// node on a candidate-prefix path, level by level in BFS (= lexicographic)
// order, which is the binder order of prep_init (mastic.py:263-275).
static int build_tree(mastic_ctx* c, const uint8_t* enc, size_t len, Tree** out) {
    std::vector<uint8_t> keyv(enc, enc + len);
    auto it = c->trees.find(keyv);
    if (it != c->trees.end()) {
        *out = it->second;
        return 0;
    }
    Tree* t = new Tree();
    std::string perr;
    const int prc = tree_parse(c->p.bits, enc, len, t, &perr);
    if (prc != TREE_OK) {
        delete t;
        return fail(c, prc == TREE_ENOMEM ? MASTIC_ENOMEM : MASTIC_EINVAL, "%s", perr.c_str());
    }
    const size_t total = t->nodes;
    const size_t npar = t->parent_node.size();
    // one device allocation and one upload: [child_path | child_exp | child_pfx | parent_node]
    const size_t o_exp = total * 32, o_pfx = o_exp + total * 4, o_par = o_pfx + total * 4;
    const size_t bytes = o_par + std::max<size_t>(npar, 1) * 4;
    if (!t->dev.ensure(bytes)) {
        delete t;
        return fail(c, MASTIC_ENOMEM, "out of device memory (tree)");
    }
    uint8_t* d = t->dev.as<uint8_t>();
    t->d_path = (uint32_t*)d;
    t->d_exp = (int32_t*)(d + o_exp);
    t->d_pfx = (int32_t*)(d + o_pfx);
    t->d_parent = (int32_t*)(d + o_par);
    // staged through a pinned buffer and copied on the main stream (the
    // kernels that read the tree queue behind it); the previous upload must
    // have left the staging buffer first
    bool staged = false;
    if (c->tree_ev || hipEventCreateWithFlags(&c->tree_ev, hipEventDisableTiming) == hipSuccess) {
        if (c->tree_stage_bytes && hipEventSynchronize(c->tree_ev) != hipSuccess) {
            delete t;
            return fail(c, MASTIC_EHIP, "tree upload failed");
        }
        if (c->tree_stage_bytes < bytes) {
            if (c->tree_stage) (void)hipHostFree(c->tree_stage);
            c->tree_stage = nullptr;
            c->tree_stage_bytes = 0;
            const size_t want = std::max(bytes, (size_t)4 << 20);
            if (hipHostMalloc(&c->tree_stage, want, hipHostMallocDefault) == hipSuccess)
                c->tree_stage_bytes = want;
            else
                (void)hipGetLastError();
        }
        if (c->tree_stage_bytes >= bytes) {
            uint8_t* h = (uint8_t*)c->tree_stage;
            std::memcpy(h, t->child_path.data(), total * 32);
            std::memcpy(h + o_exp, t->child_exp.data(), total * 4);
            std::memcpy(h + o_pfx, t->child_pfx.data(), total * 4);
            if (npar) std::memcpy(h + o_par, t->parent_node.data(), npar * 4);
            if (hipMemcpyAsync(d, h, bytes, hipMemcpyHostToDevice, c->stream) != hipSuccess ||
                hipEventRecord(c->tree_ev, c->stream) != hipSuccess) {
                delete t;
                return fail(c, MASTIC_EHIP, "tree upload failed");
            }
            staged = true;
        }
    }
    if (!staged) {  // no pinned memory: synchronous uploads from the host vectors
        hipError_t e1 = hipMemcpy(t->d_path, t->child_path.data(), total * 32, hipMemcpyHostToDevice);
        hipError_t e2 = hipMemcpy(t->d_exp, t->child_exp.data(), total * 4, hipMemcpyHostToDevice);
        hipError_t e3 = hipMemcpy(t->d_pfx, t->child_pfx.data(), total * 4, hipMemcpyHostToDevice);
        hipError_t e4 = npar ? hipMemcpy(t->d_parent, t->parent_node.data(), npar * 4, hipMemcpyHostToDevice)
                             : hipSuccess;
        if (e1 != hipSuccess || e2 != hipSuccess || e3 != hipSuccess || e4 != hipSuccess) {
            delete t;
            return fail(c, MASTIC_EHIP, "tree upload failed");
        }
    }
    if (c->trees.size() > 64) {
        // queued kernels may still read the cached trees: their device
        // buffers are retired (freed at the next idle point of the ctx's
        // streams, mastic_ctx::bury), not freed here
        for (auto& kv : c->trees) {
            DevBuf& b = kv.second->dev;
            if (b.p && b.own) c->graveyard.push_back(b.p);
            b.p = nullptr;
            b.bytes = 0;
            delete kv.second;
        }
        c->trees.clear();
    }
    c->trees[keyv] = t;
    *out = t;
    return 0;
}

// ---------------------------------------------------------------- work layout
struct WorkLayout {
    size_t words = 0;  // per report (plane count)
    size_t key, nonce, cw_seed, cw_ctrl, cw_w, cw_proof, lps, seed, peer, rk_ext, rk_conv, sp_onehot, sp_payload,
        rootsum, beta, eval_proof, proof, qr, jr, jr_part, jr_seed, verifier, status, cs[2], fr_w[2], onehot[3],
        payload[3];
};
static constexpr int NSLOT = 3;  // level buffers in flight between eval and absorb

static WorkLayout work_layout(const McParams& p, const Tree* t) {
    WorkLayout w;
    size_t o = 0;
    auto take = [&](size_t n) {
        size_t r = o;
        o += n;
        return r;
    };
    const size_t wl = (size_t)p.value_len * p.w32;
    w.key = take(4);
    w.nonce = take(4);
    w.cw_seed = take((size_t)p.bits * 4);
    w.cw_ctrl = take(p.bits);
    w.cw_w = take((size_t)p.bits * wl);
    w.cw_proof = take((size_t)p.bits * 8);
    w.lps = take((size_t)p.proof_len * p.w32);
    w.seed = take(8);
    w.peer = take(8);
    w.rk_ext = take(44);
    w.rk_conv = take(44);
    w.sp_onehot = take(50);
    w.sp_payload = take(50);
    w.rootsum = take(wl);
    w.beta = take(wl);
    w.eval_proof = take(8);
    w.proof = take((size_t)p.proof_len * p.w32);
    w.qr = take((size_t)p.query_rand_len * p.w32);
    w.jr = take((size_t)std::max(p.joint_rand_len, 1) * p.w32);
    w.jr_part = take(8);
    w.jr_seed = take(8);
    w.verifier = take((size_t)p.verifier_len * p.w32);
    w.status = take(1);
    for (int s = 0; s < 2; s++) {
        w.cs[s] = take((size_t)t->max_level_nodes * 5);
        w.fr_w[s] = take((size_t)std::max(t->max_exp, 1) * wl);
    }
    for (int k = 0; k < NSLOT; k++) {
        w.onehot[k] = take((size_t)t->max_level_nodes * 8);
        w.payload[k] = take((size_t)t->max_parents * wl);
    }
    w.words = o;
    return w;
}

static Planes make_planes(uint32_t* base, const WorkLayout& w, int n, int stride) {
    Planes pl;
    pl.n = n;
    pl.stride = stride;
    auto P = [&](size_t off) { return base + off * stride; };
    pl.key = P(w.key);
    pl.nonce = P(w.nonce);
    pl.cw_seed = P(w.cw_seed);
    pl.cw_ctrl = P(w.cw_ctrl);
    pl.cw_w = P(w.cw_w);
    pl.cw_proof = P(w.cw_proof);
    pl.lps = P(w.lps);
    pl.seed = P(w.seed);
    pl.peer = P(w.peer);
    pl.rk_ext = P(w.rk_ext);
    pl.rk_conv = P(w.rk_conv);
    pl.sp_onehot = P(w.sp_onehot);
    pl.sp_payload = P(w.sp_payload);
    pl.rootsum = P(w.rootsum);
    pl.beta = P(w.beta);
    pl.eval_proof = P(w.eval_proof);
    pl.proof = P(w.proof);
    pl.qr = P(w.qr);
    pl.jr = P(w.jr);
    pl.jr_part = P(w.jr_part);
    pl.jr_seed = P(w.jr_seed);
    pl.verifier = P(w.verifier);
    pl.status = (int32_t*)P(w.status);
    return pl;
}

static hipEvent_t get_sync_event(mastic_ctx* c, size_t i) {
    while (c->sync_ev.size() <= i) {
        hipEvent_t e;
        if (hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess) return nullptr;
        c->sync_ev.push_back(e);
    }
    return c->sync_ev[i];
}

static hipEvent_t get_event(mastic_ctx* c, size_t i) {
    while (c->tm[c->tcur].ev.size() <= i) {
        hipEvent_t e;
        if (hipEventCreate(&e) != hipSuccess) return nullptr;
        c->tm[c->tcur].ev.push_back(e);
    }
    return c->tm[c->tcur].ev[i];
}


// ---------------------------------------------------------------- prep_init
// Parents per wave: enough waves to fill 256 CUs several times over.
static int choose_ppw(int n_parents, int groups) {
    long long per = (long long)n_parents * groups / 16384;
    return (int)std::max(1LL, std::min(per, 64LL));
}

// Parents per AES wave of the level kernel.  A level is one launch and the
// next level's launch waits for its last workgroup, so the workgroup count
// should fill whole rounds of the CUs (one workgroup per CU) with nearly full
// workgroups: pick, among 8..64 parents per wave, the count whose
// (work / (rounds x CUs)) is highest, preferring more parents per wave (fewer
// table fills) within 0.5 %.
static int choose_eval_ppw(int n_parents, int groups, int aes_waves, int n_cus) {
    if ((long long)n_parents * groups < (long long)aes_waves * 8 * n_cus) return choose_ppw(n_parents, groups * 2);
    double best_eff = -1.0;
    int best = 64;
    for (int ppw = 64; ppw >= 8; ppw--) {
        const long long gy = (n_parents + (long long)aes_waves * ppw - 1) / ((long long)aes_waves * ppw);
        const long long rounds = (groups * gy + n_cus - 1) / n_cus;
        const double work = (double)groups * n_parents / ((double)aes_waves * ppw);
        const double eff = work / ((double)rounds * n_cus);
        if (eff > best_eff + 0.005) {
            best_eff = eff;
            best = ppw;
        }
    }
    return best;
}

// Items per parent at a small level (AesArgs::split).  A workgroup's 16
// waves share its items; a parent's AES is 2 extend blocks plus nblk convert
// blocks per child (next seed + payload: 2 + 2 nblk in lockstep pairs).  With
// few parents the launch time is the workgroup's longest serial chain:
// items per wave x blocks per item.  Pick the split minimising that (each
// item recomputes the extend pair; item 0 adds the next-seed pair), fewer
// items on ties.  At 16 or more parents this is 1 (no split).
// The proof waves first compute level l-1's node proofs (2 np_prev per
// report, spread over them; ~3 AES blocks of time per Keccak-p, the ratio
// miss_proof_waves uses) and then claim items from the same LDS counter, so
// the 16 waves' capacity is reduced by that head start.
static void choose_split(int n_parents, int np_prev, int proof_waves, int nblk, int* split, int* split_blocks) {
    int best_k = 1, best_cost = 1 << 30;
    const int pw = std::max(1, proof_waves);
    const int proof_blocks = np_prev > 0 ? pw * ((2 * np_prev + pw - 1) / pw) * 3 : 0;
    for (int k = 1; k <= nblk; k++) {
        const int nb = (nblk + k - 1) / k;
        const int kk = (nblk + nb - 1) / nb;  // ranges actually non-empty
        if (kk != k) continue;
        const int chain = 2 + 2 * nb;
        // the items' waves: whole items per wave after the proof waves' head start
        const int per_wave = (n_parents * k * chain + proof_blocks + EVAL_WAVES * chain - 1) / (EVAL_WAVES * chain);
        const int cost = per_wave * chain + 2;
        if (cost < best_cost) {
            best_cost = cost;
            best_k = k;
        }
    }
    *split = best_k;
    *split_blocks = (nblk + best_k - 1) / best_k;
}

static int copy_planes(mastic_ctx* c, DevBuf& dst, size_t dst_stride, size_t dst_off, const uint32_t* src,
                       size_t src_stride, size_t n, size_t planes, hipStream_t s) {
    if (planes == 0) return 0;
    HIPCHK(c, hipMemcpy2DAsync(dst.as<uint32_t>() + dst_off, dst_stride * 4, src, src_stride * 4, n * 4, planes,
                               hipMemcpyDeviceToDevice, s));
    return 0;
}

// Proof waves of a level kernel whose node proofs are fused and overlapped
// (a frontier-cache hit, kernels.hpp fuse_ovl): the proofs' share of the work
// per parent, two Keccak-p (VALU, ~3.2k CU-cycles) against the AES of the
// extend pair, the convert seeds, both children's payload blocks and the
// parent-payload recompute, 4 + 3 nblk blocks (LDS: 2 x 133 cycles per block
// at the kernel's ~50 % LDS efficiency).  C3 (Count): 7 of 16, the c2sweep
// (Sum 255, 9 payload blocks): 3.
// ... and of a miss's fused last level: per parent also the extend pair and,
// with no recompute, 3 + 2 nblk AES blocks; the proof waves also take level
// L-1's node proofs first (2 np[L-1] of them, spread over level L's parents).
static int miss_proof_waves(const McParams& p, const mastic_ctx* c, int np_prev, int np_last, bool has_prev) {
    if (c->hit_proof_waves > 0) return c->hit_proof_waves;
    const int epb = p.field == 64 ? 2 : 1;
    const int nblk = (p.value_len + epb - 1) / epb;
    const double proofs = 2.0 + (has_prev ? 2.0 * np_prev / std::max(1, np_last) : 0.0);
    const double K = 1585.0 * proofs, A = (4.0 + 2.0 * nblk) * 532.0;
    return std::max(1, std::min(12, (int)std::lround(EVAL_WAVES * K / (K + A))));
}

static int hit_proof_waves(const McParams& p, const mastic_ctx* c) {
    if (c->hit_proof_waves > 0) return c->hit_proof_waves;
    const int epb = p.field == 64 ? 2 : 1;
    const int nblk = (p.value_len + epb - 1) / epb;
    const double K = 3170.0, A = (4.0 + 3.0 * nblk) * 532.0;
    return std::max(1, std::min(12, (int)std::lround(EVAL_WAVES * K / (K + A))));
}

// One chunk of reports [base, base + n) of a prep_init, in work area W.
// lc: the frontier cache (or null); on a hit the parents are read from
// cin (the aggregator's node slot); the last level's nodes go to cout (the
// spare slot).  tail: the stream of the chunk's last part (finalize, FLP,
// result and cache copies): the sponge stream when chunks are pipelined (the
// next chunk's evaluation, in the other half of the work arena, then
// overlaps this chunk's last sponges), else the main stream.  sev0: first
// sync event of this chunk (consecutive pipelined chunks use disjoint ones).
template <class F>
static int run_chunk(mastic_ctx* c, mastic_reports* rep, const Tree* t, const WorkLayout& wl, int agg_id,
                     size_t base, int n, int stride, size_t& evi, LevelCache* lc, bool hit, const uint32_t* cin,
                     uint32_t* cout, uint32_t* W, hipStream_t ss, hipStream_t tail, size_t sev0) {
    const McParams& p = c->p;
    Planes pl = make_planes(W, wl, n, stride);
    Result& R = c->res[agg_id];
    // A single-chunk call with the frontier cache keeps both binder sponges
    // and the root sum in the cache's planes (same stride): a hit resumes and
    // updates them in place, a miss fills them; no copies in or out.
    const bool direct = lc && base == 0 && (size_t)n == rep->n && lc->S == (size_t)stride;
    if (direct) {
        pl.sp_onehot = lc->sp.as<uint32_t>();
        pl.sp_payload = lc->sp.as<uint32_t>() + (size_t)50 * lc->S;
        pl.rootsum = lc->rootsum.as<uint32_t>();
    }
    // Every level plane (child seeds, frontier payloads, proof / payload-
    // difference ring, out shares, staged last-level payloads) is written
    // before it is read: level l reads only level l-1's nodes / expanded
    // nodes, which level l-1 wrote, and each candidate prefix is one child of
    // level L.  So only the per-report header planes (keys, correction words,
    // sponge states, FLP planes, status) are cleared -- 8 KB per report at C2
    // instead of the whole 9.7 MB work area (119 GB of fill per C2 step).  A
    // frontier-cache hit writes every header plane it reads except the
    // status plane: it clears just that.
    if (hit)
        HIPCHK(c, hipMemsetAsync(pl.status, 0, (size_t)stride * 4, c->stream));
    else {
        // Of the header, the keys, nonces and correction words (k_unpack: every
        // report row, every level the call reads) and the AES key schedules and
        // sponge states (k_setup: every row) are written in full before any
        // read, so only their padding rows are cleared; the planes between
        // (leader proof share, seeds: by aggregator and circuit) and from the
        // root sum on (accumulated root sum and FLP, result and status planes)
        // are cleared whole.  C2: 409 of 2,107 header words per report.
        // (work_layout order: key, nonce, cw_* | lps, seed, peer | rk_*, sp_* | rootsum .. status)
        HIPCHK(c, hipMemsetAsync(W + wl.lps * (size_t)stride, 0, (wl.rk_ext - wl.lps) * (size_t)stride * 4, c->stream));
        HIPCHK(c, hipMemsetAsync(W + wl.rootsum * (size_t)stride, 0, (wl.cs[0] - wl.rootsum) * (size_t)stride * 4,
                                 c->stream));
        if (stride > n)
            HIPCHK(c, hipMemset2DAsync(W + n, (size_t)stride * 4, 0, (size_t)(stride - n) * 4, wl.lps, c->stream));
        // level 0 reads its parent (the root) payload from fr_w[1]: zeros
        HIPCHK(c, hipMemsetAsync(W + wl.fr_w[1] * (size_t)stride, 0, (size_t)p.value_len * p.w32 * stride * 4, c->stream));
    }
    const size_t ps = mc_public_share_size(p), is = mc_input_share_size(p, agg_id);
    const uint8_t* ins = agg_id == 0 ? rep->in0.as<uint8_t>() : rep->in1.as<uint8_t>();
    const PrefixState* pfx = (const PrefixState*)c->pfx.p;
    {
        const uint8_t* pub = rep->pub.as<uint8_t>() + ps * base;
        const uint8_t* in_b = ins + is * base;
        const int l_lo = hit ? t->L - 1 : 0, l_hi = t->L + 1;  // a hit recomputes level L-1's payloads: its CW
        // Rows of >= 16 KB to unpack per report (C4, C5), 8-byte aligned
        // (BITS a multiple of 32): the correction words and the leader proof
        // share, the bulk of a report's bytes, go through coalesced row tiles;
        // k_unpack keeps the nonce, key, control bits and seeds.  Same-box A/B
        // (profiles/r05_v37_ab_row_tile_unpack.txt): C5 +2.2 %, C4 +0.5 %;
        // the 1M sweep's rows (<= 5.9 KB) gained nothing in wall time (+0.1 %)
        // while its level kernels, started earlier under the previous chunk's
        // sponges, measured 1.3 % longer, so small rows keep one lane per report.
        const size_t nctrl = (2 * (size_t)p.bits + 7) / 8;
        const size_t row_bytes = (size_t)(l_hi - l_lo) * (16 + (size_t)p.value_len * p.enc + 32) +
                                 (agg_id == 0 ? (size_t)p.proof_len * p.enc : 0);
        // (grid y of every row-tile launch below: 64 words per workgroup row)
        const size_t max_words = std::max<size_t>((size_t)p.value_len * p.w32 * (l_hi - l_lo),
                                                  agg_id == 0 ? (size_t)p.proof_len * p.w32 : 0);
        const bool tiles = row_bytes >= 16384 && (((uintptr_t)pub | (uintptr_t)in_b | ps | is | nctrl) & 7) == 0 &&
                           (max_words + 63) / 64 < 65535;
        hipLaunchKernelGGL(k_unpack, dim3((n + 255) / 256), dim3(256), 0, c->stream, p, pl, agg_id,
                           rep->nonces.as<uint8_t>() + 16 * base, pub, in_b, l_lo, l_hi, tiles ? 1 : 0);
        if (tiles) {
            const int wlw_ = p.value_len * p.w32, nl = l_hi - l_lo;
            auto rows = [&](const uint8_t* src, size_t row_bytes, int nwords, uint32_t* dst) {
                if (nwords <= 0) return;
                hipLaunchKernelGGL(k_rows_to_planes, dim3((unsigned)((n + 63) / 64), (unsigned)((nwords + 63) / 64)),
                                   dim3(256), 0, c->stream, src, row_bytes, n, nwords, dst, stride);
            };
            const uint8_t* seg = pub + nctrl;
            rows(seg + 16 * (size_t)l_lo, ps, 4 * nl, pl.cw_seed + (size_t)4 * l_lo * stride);
            seg += 16 * (size_t)p.bits;
            rows(seg + (size_t)l_lo * p.value_len * p.enc, ps, wlw_ * nl, pl.cw_w + (size_t)wlw_ * l_lo * stride);
            seg += (size_t)p.bits * p.value_len * p.enc;
            rows(seg + 32 * (size_t)l_lo, ps, 8 * nl, pl.cw_proof + (size_t)8 * l_lo * stride);
            if (agg_id == 0) rows(in_b + 16, is, p.proof_len * p.w32, pl.lps);
        }
        HIPCHK(c, hipGetLastError());
    }
    const bool whole = base == 0 && (size_t)n == rep->n && W == c->work.p;
    const bool rk_ok = hit && whole && c->rk.valid && c->rk.rep_id == rep->id && c->rk.rep_gen == rep->generation() &&
                       c->rk.n == (size_t)n && c->rk.stride == stride && c->rk.W == (const void*)W &&
                       c->rk.pfx_key == c->pfx_key;
    if (!rk_ok) {
        hipLaunchKernelGGL(k_setup, dim3((stride + 255) / 256), dim3(256), 0, c->stream, pl, pfx, hit ? 0 : 1);
        c->rk.valid = whole;
        c->rk.rep_id = rep->id;
        c->rk.rep_gen = rep->generation();
        c->rk.n = (size_t)n;
        c->rk.stride = stride;
        c->rk.W = (const void*)W;
        c->rk.pfx_key = c->pfx_key;
    }
    HIPCHK(c, hipGetLastError());

    const int groups = (n + 63) / 64;  // report groups (rows beyond n are padding)
    const int wlw = p.value_len * p.w32;
    int f_oh = c->pfx_f[PFX_ONEHOT], f_pl = c->pfx_f[PFX_PAYLOAD];
    auto plane = [&](size_t off) { return W + off * (size_t)stride; };
    // Per level l, on two streams:
    //   stream   k_eval_aes(l): AES of level l (12 waves per workgroup) and
    //            the node proofs of level l-1 (4 proof waves per workgroup)
    //   stream2  k_absorb(l-1): binder sponges over level l-1's proofs and
    //            payload differences, after eval_aes(l)
    // so the sponges of one level overlap the evaluation of the next.  The
    // last level's proofs come from a k_node_proof launch.  Buffers: child
    // seeds 2 slots; proof / payload 3 slots (eval_aes(l) writes payload(l)
    // and proofs(l-1), so it waits absorb(l-3)).  Timing: one (eval, proof,
    // absorb) event triplet per step of the loop below.
    size_t sev = sev0;
    std::vector<hipEvent_t> abs_done(t->L + 1);
    // tiled level buffers (kernels.hpp AbsorbArgs): words per report group
    // (MASTIC_BINDER_TILED=0: plane layout, i.e. group stride 64, row stride = stride)
    const int oh_gstride = c->binder_tiled ? t->max_level_nodes * 8 * 64 : 64;
    const int pay_gstride = c->binder_tiled ? t->max_parents * wlw * 64 : 64;
    const int bin_rstride = c->binder_tiled ? 64 : stride;
    // level binder buffers: the ring slots (with the frontier cache too: a
    // hit resumes both sponges from their cached states, so no level's
    // proofs or payload differences outlive the call)
    auto oh_buf = [&](int lv) -> uint32_t* { return plane(wl.onehot[lv % NSLOT]); };
    auto pay_buf = [&](int lv) -> uint32_t* { return plane(wl.payload[lv % NSLOT]); };
    auto oh_gs = [&](int) -> int { return oh_gstride; };
    auto pay_gs = [&](int) -> int { return pay_gstride; };
    // Sponges which0 .. which0 + nwh - 1 (0 one-hot, 1 payload) of level lv on
    // stream `as` after `ready`; *done marks their end.
    const bool pair = c->absorb_mode == 2 || (c->absorb_mode == 0 && (size_t)n < c->absorb_single_min);
    auto launch_sponges = [&](int lv, int which0, int nwh, hipEvent_t ready, hipEvent_t e4, hipEvent_t e5,
                              hipStream_t as, hipEvent_t* done) -> int {
        AbsorbArgs ab;
        ab.which0 = which0;
        ab.seg[0] = oh_buf(lv);
        ab.gstride[0] = oh_gs(lv);
        ab.nbytes[0] = 2 * t->n_parents[lv] * 32;
        ab.f[0] = f_oh;
        ab.seg[1] = pay_buf(lv);
        ab.gstride[1] = pay_gs(lv);
        ab.rstride = bin_rstride;
        ab.nbytes[1] = lv > 0 ? t->n_parents[lv] * wlw * 4 : 0;
        ab.f[1] = f_pl;
        ab.prio = c->absorb_prio;
        ab.dbg = c->absorb_dbg;
        if (as != c->stream) HIPCHK(c, hipStreamWaitEvent(as, ready, 0));
        if (e4) HIPCHK(c, hipEventRecord(e4, as));
        if (c->dbg_skip & 4) {
            // timing experiments only: no binder sponges (results wrong)
        } else if (pair)
            hipLaunchKernelGGL(k_absorb_pair,
                               dim3((groups * 64 * 2 + c->absorb_threads - 1) / c->absorb_threads, (unsigned)nwh),
                               dim3(c->absorb_threads), c->absorb_lds, as, pl, ab);
        else
            hipLaunchKernelGGL(k_absorb, dim3((groups * 64 + 255) / 256, (unsigned)nwh), dim3(256), c->absorb_lds, as,
                               pl, ab);
        if (e5) HIPCHK(c, hipEventRecord(e5, as));
        HIPCHK(c, hipGetLastError());
        *done = get_sync_event(c, sev++);
        HIPCHK(c, hipEventRecord(*done, as));
        // measurement schedule (mastic_set_serial_sponges): the main stream waits
        // for this launch, so it runs alone on the chip (standalone sponge rate)
        if (c->serial_sponges && as != c->stream) HIPCHK(c, hipStreamWaitEvent(c->stream, *done, 0));
        if (which0 == 0) f_oh = (f_oh + ab.nbytes[0]) % KECCAK_RATE;
        if (which0 + nwh > 1) f_pl = (f_pl + ab.nbytes[1]) % KECCAK_RATE;
        return 0;
    };
    // both sponges of level lv (the default schedule)
    std::vector<hipEvent_t> pl_done(t->L + 1, nullptr);  // split schedule: payload sponge of each level
    auto launch_absorb = [&](int lv, hipEvent_t ready, hipEvent_t e4, hipEvent_t e5, hipStream_t as) -> int {
        return launch_sponges(lv, 0, 2, ready, e4, e5, as, &abs_done[lv]);
    };
    // Split schedule (single-chunk misses, MASTIC_SPLIT_SPONGES): level l's
    // payload differences are complete after eval(l), so its payload sponge
    // starts then, on the third stream, while its one-hot sponge still waits
    // for level l's node proofs (eval(l+1)'s proof waves).  The payload chain
    // -- the long one at C4 / C5 -- then runs a level earlier and leaves a
    // shorter tail after the last level.
    // Measured (profiles/r04_v23_ab_split_sponges.txt): C5 +1.4 %, C4 +0.6 %,
    // C2 -0.5 %, c2sweep -0.9 % -- so by default for Field128 only, whose
    // payload messages (VALUE_LEN x 16 B per parent) make that chain long.
    const bool split_on = c->split_sponges < 0 ? p.field == 128 : c->split_sponges > 0;
    const bool split = split_on && !hit && tail == c->stream && ss == c->stream2;
    // cache planes <-> work planes of this chunk (columns base .. base + n)
    auto from_cache = [&](uint32_t* dst, const uint32_t* src, size_t planes) -> int {
        HIPCHK(c, hipMemcpy2DAsync(dst, (size_t)stride * 4, src + base, lc->S * 4, (size_t)n * 4, planes,
                                   hipMemcpyDeviceToDevice, c->stream));
        return 0;
    };
    auto to_cache = [&](uint32_t* dst, const uint32_t* src, size_t planes) -> int {
        HIPCHK(c, hipMemcpy2DAsync(dst + base, lc->S * 4, src, (size_t)stride * 4, (size_t)n * 4, planes,
                                   hipMemcpyDeviceToDevice, tail));
        return 0;
    };
    if (hit && !direct) {
        // levels 0..L-1 from the cache.  The binder messages are BFS-ordered
        // (mastic.py:263-275), so the cached call's message is a prefix of
        // this one's: both sponges resume from their states at the end of the
        // cached call (mid-block, unpadded; k_finalize pads a register copy).
        if (from_cache(pl.sp_onehot, lc->sp.as<uint32_t>(), 50)) return -1;
        if (from_cache(pl.sp_payload, lc->sp.as<uint32_t>() + (size_t)50 * lc->S, 50)) return -1;
        // the root sum of the cached level-0 evaluation (counter check)
        if (from_cache(pl.rootsum, lc->rootsum.as<uint32_t>(), (size_t)wlw)) return -1;
    }
    if (hit) {
        // (no timing events for the cached levels: nothing is launched for
        // them, and 6 records per level cost ~1.4 ms of host time at L = 255)
        for (int lv = 0; lv < t->L; lv++) {
            f_oh = (f_oh + 2 * t->n_parents[lv] * 32) % KECCAK_RATE;
            f_pl = (f_pl + (lv > 0 ? t->n_parents[lv] * wlw * 4 : 0)) % KECCAK_RATE;
        }
    }
    // the last level's node proofs in the level kernel (after each workgroup's
    // parents) instead of a k_node_proof launch: cache hits, and with
    // MASTIC_FUSE_PROOFS=2 cache-on misses too (whole parents only)
    // A miss's last level is fused too when the frontier cache is on (the
    // sweeps: c2sweep +1 %, its level kernels -4 %), not without it (C2 -1.7 %,
    // C5 -0.9 %: the FC kernel's 128 VGPRs leave no room for the previous
    // level's sponge waves beside it; profiles/r04_v21_ab_fused_last_miss.txt)
    const bool fuse_last = hit ? c->fuse_proofs >= 1
                               : ((lc && (c->fuse_proofs == 2 || (c->fuse_proofs >= 1 && c->fuse_last_miss_fc))) ||
                                  (c->fuse_last_miss && c->fuse_proofs >= 1));
    // The last level's sponges: on the main stream for a hit that runs as one
    // chunk (nothing to overlap them with: the next work on the main stream
    // needs them; the cross-stream event round trip cost ~0.08 ms per call),
    // else on the sponge stream after the level's earlier sponges.
    const hipStream_t last_as = (hit && tail == c->stream && c->hit_absorb_main) ? c->stream : ss;
    for (int l = hit ? t->L : 0; l <= t->L; l++) {
        const int np_ = t->n_parents[l];
        if (!hit && l >= NSLOT) {
            HIPCHK(c, hipStreamWaitEvent(c->stream, abs_done[l - NSLOT], 0));
            if (split && pl_done[l - NSLOT]) HIPCHK(c, hipStreamWaitEvent(c->stream, pl_done[l - NSLOT], 0));
        }
        AesArgs a;
        a.level = l;
        a.agg_id = agg_id;
        a.n_parents = np_;
        // items per workgroup: par_waves x ppw, par_waves = the AES waves (the
        // proof waves mop up after their proofs).  MASTIC_PAR_WAVES=16 hands
        // all waves parents from the start: measured neutral on C4 and C2 and
        // 3 % slower on C5 (profiles/r02_v12_ab_level_kernel.json)
        const int par_waves = c->par_waves > 0 ? c->par_waves : EVAL_WAVES - c->proof_waves;
        // small levels: parents split into block-range items (AesArgs::split);
        // not at the last level (out shares, frontier-cache staging) nor on a hit
        a.split = 1;
        a.split_blocks = 0;
        {
            const int epb = p.field == 64 ? 2 : 1;
            const int nblk = (p.value_len + epb - 1) / epb;
            a.split_blocks = nblk;
            // (<= 32 parents: their pass-0 flags live in the workgroup's sync words)
            if (!hit && l < t->L && c->small_split && np_ <= 32 && !(c->dbg_skip & 2))
                choose_split(np_, l > 0 ? t->n_parents[l - 1] : 0, c->proof_waves, nblk, &a.split,
                             &a.split_blocks);
        }
        const int n_items = np_ * a.split;
        a.ppw = choose_eval_ppw(n_items, groups, par_waves, c->n_cus);
        // a split level keeps all items of a report group in one workgroup
        // (the fix-up pass needs every item of a parent stored): gy = 1
        if (a.split > 1) a.ppw = (n_items + par_waves - 1) / par_waves;
        a.parent_node = t->d_parent + t->poff[l];
        a.child_exp = t->d_exp + t->off[l];
        a.child_pfx = t->d_pfx + t->off[l];
        a.cs_in = hit ? cin + base : plane(wl.cs[(l + 1) & 1]);
        a.cs_out = plane(wl.cs[l & 1]);
        a.fr_w_in = plane(wl.fr_w[(l + 1) & 1]);
        a.in_stride = hit ? (int)lc->S : stride;
        a.fr_w_out = plane(wl.fr_w[l & 1]);
        a.payload = pay_buf(l);
        a.out = R.out.as<uint32_t>() + base;  // columns base .. base + n of the result planes
        a.out_stride = (int)R.stride;
        a.force_slow_blk = c->force_slow_blk;
        // frontier cache: stage this level's convert seeds (last level); on a
        // hit recompute the parents' payloads from the cached ones into the
        // (otherwise unused) parent-payload planes
        a.cache_out = (lc && l == t->L) ? cout + base : nullptr;
        a.cache_stride = lc ? (int)lc->S : 0;
        a.wp_buf = plane(wl.fr_w[(l + 1) & 1]);
        a.recompute_wp = hit ? 1 : 0;
        const bool fuse = fuse_last && l == t->L;
        a.fuse_proofs = fuse ? (c->fuse_proofs == 3 ? 3 : 1) : 0;
        a.cur_path_bytes = (l + 1 + 7) / 8;
        a.cur_child_path = t->d_path + t->off[l] * 8;
        a.cur_onehot = oh_buf(l);
        a.aes_waves = EVAL_WAVES - c->proof_waves;
        if (fuse && a.fuse_proofs == 1)
            a.aes_waves = EVAL_WAVES - (hit ? hit_proof_waves(p, c) : miss_proof_waves(p, c, t->n_parents[l - 1 < 0 ? 0 : l - 1],
                                                                                      np_, l > 0));
        a.par_waves = par_waves;
        a.proof_prio = c->proof_prio;
        a.aes_prio = c->aes_prio;
        a.dbg_skip = c->dbg_skip;
        const int gy = (n_items + a.par_waves * a.ppw - 1) / (a.par_waves * a.ppw);
        a.pv_level = l - 1;
        a.pv_nodes = (l > 0 && !hit) ? 2 * t->n_parents[l - 1] : 0;  // hit: level L-1's proofs are cached
        const int pw = EVAL_WAVES - a.aes_waves;  // proof waves of this launch
        a.pv_npw = (a.pv_nodes + gy * pw - 1) / (gy * pw);
        a.pv_path_bytes = (l + 7) / 8;
        a.pv_child_path = l > 0 ? t->d_path + t->off[l - 1] * 8 : nullptr;
        a.pv_onehot = l > 0 ? oh_buf(l - 1) : nullptr;
        a.oh_gstride = l > 0 ? oh_gs(l - 1) : oh_gstride;
        a.pay_gstride = pay_gs(l);
        a.bin_rstride = bin_rstride;
        a.np = (const PrefixState*)c->pfx.p + PFX_NODE;
        a.np_f = c->pfx_f[PFX_NODE];
        dim3 grid(groups, gy);
        hipEvent_t e0 = get_event(c, evi++), e1 = get_event(c, evi++);
        hipEvent_t e2 = get_event(c, evi++), e3 = get_event(c, evi++);
        hipEvent_t e4 = get_event(c, evi++), e5 = get_event(c, evi++);
        HIPCHK(c, hipEventRecord(e0, c->stream));
        // the frontier-cache variant only where its features are used: the
        // last level (convert seeds staged for the cache) and a hit (parent
        // payloads recomputed, fused proofs); a miss's other levels run the
        // plain kernel (the variant's uniform branches and extra spills cost
        // a few per cent)
        if ((lc && (hit || l == t->L || c->fc_all)) || fuse)
            hipLaunchKernelGGL((k_eval_aes<F, true, true>), grid, dim3(64 * EVAL_WAVES), EVAL_LDS_BYTES, c->stream,
                               p, pl, a);
        else if (a.split > 1 && l == 0)
            hipLaunchKernelGGL((k_eval_aes<F, true, false, true>), grid, dim3(64 * EVAL_WAVES), EVAL_LDS_BYTES,
                               c->stream, p, pl, a);
        else if (a.split > 1)
            hipLaunchKernelGGL((k_eval_aes<F, false, false, true>), grid, dim3(64 * EVAL_WAVES), EVAL_LDS_BYTES,
                               c->stream, p, pl, a);
        else if (l == 0 || l == t->L)
            hipLaunchKernelGGL((k_eval_aes<F, true, false>), grid, dim3(64 * EVAL_WAVES), EVAL_LDS_BYTES, c->stream,
                               p, pl, a);
        else
            hipLaunchKernelGGL((k_eval_aes<F, false, false>), grid, dim3(64 * EVAL_WAVES), EVAL_LDS_BYTES, c->stream,
                               p, pl, a);
        HIPCHK(c, hipEventRecord(e1, c->stream));
        HIPCHK(c, hipGetLastError());
        HIPCHK(c, hipEventRecord(e2, c->stream));
        HIPCHK(c, hipEventRecord(e3, c->stream));
        hipEvent_t aes_done = get_sync_event(c, sev++);
        HIPCHK(c, hipEventRecord(aes_done, c->stream));
        if (split && l > 0) {
            // payload(l) now, one-hot(l-1) after the proofs this launch made
            if (launch_sponges(l, 1, 1, aes_done, e4, e5, c->stream3, &pl_done[l])) return -1;
            if (launch_sponges(l - 1, 0, 1, aes_done, nullptr, nullptr, ss, &abs_done[l - 1])) return -1;
        } else if (l > 0 && !hit) {
            if (launch_absorb(l - 1, aes_done, e4, e5, ss)) return -1;
        } else {
            if (c->sponge_delay_us > 0) {
                // test hook: the sponge stream is still busy when these (empty)
                // marks are recorded there; nothing on the main stream waits for them
                const unsigned long long ticks =
                    (unsigned long long)c->sponge_delay_us * (unsigned long long)c->wall_khz / 1000;
                c->sponge_delay_us = 0;
                hipLaunchKernelGGL(k_spin, dim3(1), dim3(64), 0, ss, ticks);
                HIPCHK(c, hipGetLastError());
            }
            HIPCHK(c, hipEventRecord(e4, ss));
            HIPCHK(c, hipEventRecord(e5, ss));
        }
    }
    if (fuse_last) {
        // the last level's proofs came from the level kernel's AES waves: its sponges
        const int l = t->L;
        hipEvent_t e0 = get_event(c, evi++), e1 = get_event(c, evi++);
        hipEvent_t e2 = get_event(c, evi++), e3 = get_event(c, evi++);
        hipEvent_t e4 = get_event(c, evi++), e5 = get_event(c, evi++);
        HIPCHK(c, hipEventRecord(e0, c->stream));
        HIPCHK(c, hipEventRecord(e1, c->stream));
        HIPCHK(c, hipEventRecord(e2, c->stream));
        HIPCHK(c, hipEventRecord(e3, c->stream));
        hipEvent_t np_done = get_sync_event(c, sev++);
        HIPCHK(c, hipEventRecord(np_done, c->stream));
        if (split ? launch_sponges(l, 0, 1, np_done, e4, e5, last_as, &abs_done[l])
                  : launch_absorb(l, np_done, e4, e5, last_as))
            return -1;
    } else {
        // the last level's node proofs, then its sponges
        const int l = t->L;
        const int nn = 2 * t->n_parents[l];
        ProofArgs pa;
        pa.level = l;
        pa.n_nodes = nn;
        pa.npw = choose_ppw(nn, groups);
        pa.path_bytes = (l + 1 + 7) / 8;
        pa.child_path = t->d_path + t->off[l] * 8;
        pa.cs = plane(wl.cs[l & 1]);
        pa.onehot = oh_buf(l);
        pa.oh_gstride = oh_gs(l);
        pa.bin_rstride = bin_rstride;
        pa.np = (const PrefixState*)c->pfx.p + PFX_NODE;
        pa.f = c->pfx_f[PFX_NODE];
        hipEvent_t e0 = get_event(c, evi++), e1 = get_event(c, evi++);
        hipEvent_t e2 = get_event(c, evi++), e3 = get_event(c, evi++);
        hipEvent_t e4 = get_event(c, evi++), e5 = get_event(c, evi++);
        HIPCHK(c, hipEventRecord(e0, c->stream));
        HIPCHK(c, hipEventRecord(e1, c->stream));
        HIPCHK(c, hipEventRecord(e2, c->stream));
        hipLaunchKernelGGL(k_node_proof, dim3(groups, (nn + 4 * pa.npw - 1) / (4 * pa.npw)), dim3(256), 0,
                           c->stream, p, pl, pa);
        HIPCHK(c, hipEventRecord(e3, c->stream));
        HIPCHK(c, hipGetLastError());
        hipEvent_t np_done = get_sync_event(c, sev++);
        HIPCHK(c, hipEventRecord(np_done, c->stream));
        if (split ? launch_sponges(l, 0, 1, np_done, e4, e5, last_as, &abs_done[l])
                  : launch_absorb(l, np_done, e4, e5, last_as))
            return -1;
    }
    hipEvent_t flp_done = nullptr;
    if (t->weight_check) {
        // The FLP randomness and query (mastic.py:234-256) read only header
        // planes and level 0's root sum: on their own stream once the last
        // level kernel is done, beside the last level's sponges (a few
        // latency-bound chains that leave most of the chip idle: C5's last
        // payload chain runs ~34 ms) instead of after them.  (Right after
        // level 0 they slowed the level kernels beside them by as much as
        // they saved: C4 -1.8 %, profiles/r05_v36_ab_flp_side_stream.txt.)
        hipEvent_t lv_done = get_sync_event(c, sev++);
        HIPCHK(c, hipEventRecord(lv_done, c->stream));
        HIPCHK(c, hipStreamWaitEvent(c->stream4, lv_done, 0));
        FlpArgs fl{agg_id, t->L};
        hipLaunchKernelGGL(k_flp_rand<F>, dim3((stride + 255) / 256), dim3(256), 0, c->stream4, p, pl, fl, pfx);
        hipLaunchKernelGGL(k_flp_query<F>, dim3((stride + 255) / 256), dim3(256), 0, c->stream4, p, pl,
                           flp_consts<F>(p));
        HIPCHK(c, hipGetLastError());
        flp_done = get_sync_event(c, sev++);
        HIPCHK(c, hipEventRecord(flp_done, c->stream4));
    }
    if (tail != last_as) HIPCHK(c, hipStreamWaitEvent(tail, abs_done[t->L], 0));
    if (split && pl_done[t->L]) HIPCHK(c, hipStreamWaitEvent(tail, pl_done[t->L], 0));
    FinalArgs fa{agg_id, f_oh, f_pl};
    hipLaunchKernelGGL(k_finalize<F>, dim3((stride + 255) / 256), dim3(256), 0, tail, p, pl, fa, pfx);
    HIPCHK(c, hipGetLastError());
    // the status, verifier and joint-rand planes copied below are the FLP's
    if (flp_done) HIPCHK(c, hipStreamWaitEvent(tail, flp_done, 0));
    if (lc && !direct) {
        // frontier cache for the next level (the last level's nodes are in the
        // spare slot already, written by its level kernel): the root sum
        if (!hit && to_cache(lc->rootsum.as<uint32_t>(), pl.rootsum, (size_t)wlw)) return -1;
        // both sponges after levels 0..L (stream waited for abs_done[L] above)
        if (to_cache(lc->sp.as<uint32_t>(), pl.sp_onehot, 50)) return -1;
        if (to_cache(lc->sp.as<uint32_t>() + (size_t)50 * lc->S, pl.sp_payload, 50)) return -1;
    }
    // results -> the agg_id slot (plane stride = all reports; the level
    // kernel wrote the out shares there)
    int rc = 0;
    rc |= copy_planes(c, R.eval_proof, R.stride, base, pl.eval_proof, stride, n, 8, tail);
    rc |= copy_planes(c, R.status, R.stride, base, (const uint32_t*)pl.status, stride, n, 1, tail);
    if (t->weight_check) {
        rc |= copy_planes(c, R.verifier, R.stride, base, pl.verifier, stride, n, (size_t)p.verifier_len * p.w32,
                          tail);
        if (p.joint_rand_len > 0) {
            rc |= copy_planes(c, R.jr_part, R.stride, base, pl.jr_part, stride, n, 8, tail);
            rc |= copy_planes(c, R.jr_seed, R.stride, base, pl.jr_seed, stride, n, 8, tail);
        }
    }
    return rc;
}

static uint64_t default_budget(mastic_ctx* c) {
    if (c->budget) return c->budget;
    size_t freeb = 0, total = 0;
    if (hipMemGetInfo(&freeb, &total) != hipSuccess) return 1ull << 30;
    // work buffers are the only large allocation (C2: ~8.6 MB per report);
    // one chunk per batch keeps one binder-sponge chain per prep_init
    return (uint64_t)(freeb * 0.75);
}

extern "C" int mastic_prep_init(mastic_ctx* c, mastic_reports* rep, const uint8_t* verify_key, size_t vk_len,
                                const uint8_t* app_ctx, size_t ctx_len, int agg_id, const uint8_t* enc_agg_param,
                                size_t agg_param_len) {
    DeviceScope ds_(c);
    if (!c || !rep || rep->ctx != c) return fail(c, MASTIC_EINVAL, "bad ctx/reports");
    if (agg_id != 0 && agg_id != 1) return fail(c, MASTIC_EINVAL, "invalid aggregator ID");
    if ((agg_id == 0 && !rep->in0.p) || (agg_id == 1 && !rep->in1.p))
        return fail(c, MASTIC_EINVAL, "reports hold no input shares for this aggregator");
    if (!verify_key && vk_len) return fail(c, MASTIC_EINVAL, "verify key required");
    static const uint8_t empty_vk[1] = {0};
    if (!verify_key) verify_key = empty_vk;
    c->tcur = agg_id;
    Tree* t = nullptr;
    int rc = build_tree(c, enc_agg_param, agg_param_len, &t);
    if (rc) return rc;
    if ((rc = build_prefixes(c, app_ctx, ctx_len, verify_key, vk_len))) return rc;
    const McParams& p = c->p;
    WorkLayout wl = work_layout(p, t);
    const size_t n = rep->n;
    Result& R = c->res[agg_id];
    R.ready = false;
    R.n = n;
    R.stride = round_up(std::max<size_t>(n, 1), 64);
    R.weight_check = t->weight_check;
    R.n_prefixes = t->n_prefixes;
    const size_t S = R.stride;
    // a result buffer that must grow retires the old one to the graveyard
    // (freed at the next idle point) instead of freeing it here: hipFree
    // waits for the whole device, i.e. for the other aggregator's queued call
    auto rgrow = [&](DevBuf& d, size_t want) {
        if (want <= d.bytes && d.p) return true;
        const size_t old = d.bytes;
        if (d.p && d.own) c->graveyard.push_back(d.p);
        d.p = nullptr;
        d.bytes = 0;
        d.own = true;
        if (!c->inject_alloc_failure() && (d.ensure(std::max(want, old + old / 2)) || d.ensure(want))) return true;
        // HBM is held by the work arena (sized to the budget when the results
        // were smaller) and by retired buffers: once the queued work on all
        // three streams is done, free both and retry; the arena is re-allocated
        // below, within what is left (a 2M-report sweep's out shares reach 32 GB
        // per aggregator)
        if (!c->idle()) return false;
        c->bury();
        c->work.release();
        c->rk.valid = false;
        return d.ensure(want);
    };
    if (!rgrow(R.eval_proof, S * 8 * 4) || !rgrow(R.status, S * 4) ||
        !rgrow(R.out, S * 4 * std::max<size_t>(1, (size_t)t->n_prefixes * (1 + p.output_len) * p.w32)) ||
        !rgrow(R.verifier, S * 4 * (size_t)p.verifier_len * p.w32) || !rgrow(R.jr_part, S * 32) ||
        !rgrow(R.jr_seed, S * 32))
        return fail(c, MASTIC_ENOMEM, "out of device memory (results for %zu reports)", n);
    HIPCHK(c, hipMemsetAsync(R.jr_part.p, 0, S * 32, c->stream));
    HIPCHK(c, hipMemsetAsync(R.jr_seed.p, 0, S * 32, c->stream));
    if (n == 0) {
        R.ready = true;
        return 0;
    }
    const size_t pad = (size_t)c->stride_pad;
    // frontier cache (tiled binder buffers only): decide hit / miss and size
    // the slot before the work buffer, so the HBM budget sees the cache
    LevelCache* lc = nullptr;
    bool hit = false;
    const uint32_t* cin = nullptr;  // a hit's parents: this aggregator's node slot
    uint32_t* cout = nullptr;       // the last level's nodes: the spare node slot
    std::vector<uint8_t> lkey(1, (uint8_t)vk_len);
    lkey.insert(lkey.end(), verify_key, verify_key + vk_len);
    lkey.insert(lkey.end(), app_ctx, app_ctx + ctx_len);
    if (c->frontier_cache && c->binder_tiled) {
        lc = &c->lc[agg_id];
        const size_t S1 = round_up(n, 64) + pad;
        const int L = t->L;
        hit = lc->valid && lc->rep_id == rep->id && lc->rep_gen == rep->generation() && lc->n == n && lc->S == S1 && lc->key == lkey &&
              !t->weight_check && L == lc->L + 1 && (size_t)L <= lc->n_parents.size() &&
              std::equal(t->n_parents.begin(), t->n_parents.begin() + L, lc->n_parents.begin()) &&
              // level L-1's node paths fix every level above (each level's
              // parents are the truncations of the next level's nodes), so
              // they and the node counts decide that the trees agree there
              lc->paths.size() == (t->off[L] - t->off[L - 1]) * 8 &&
              std::equal(lc->paths.begin(), lc->paths.end(), t->child_path.begin() + t->off[L - 1] * 8);
        auto retire = [&](DevBuf& b) {  // queued kernels may still read it
            if (b.p && b.own) c->graveyard.push_back(b.p);
            b.p = nullptr;
            b.bytes = 0;
        };
        if (lc->S != S1) {
            retire(lc->sp);
            retire(lc->rootsum);
            retire(lc->nd);
            lc->nodes_cap = 0;
            lc->S = S1;
        }
        if (c->spare_S != S1) {
            retire(c->fc_spare);
            c->spare_cap = 0;
            c->spare_S = S1;
        }
        const size_t wlw = (size_t)p.value_len * p.w32;
        const size_t nl = (size_t)2 * t->n_parents[L];
        // an allocation that fails first reclaims what idle streams free: the
        // retired slots and the work buffer (re-allocated below, to the budget)
        auto alloc = [&](DevBuf& b, size_t bytes) -> bool {
            if (!c->inject_alloc_failure() && b.ensure(bytes)) return true;
            if (!c->idle()) return false;
            c->bury();
            c->work.release();
            c->rk.valid = false;
            return b.ensure(bytes);
        };
        bool ok = alloc(lc->sp, 100 * S1 * 4) && alloc(lc->rootsum, wlw * S1 * 4);
        if (ok && nl > c->spare_cap) {
            // grow geometrically (a sweep's frontier widens over several
            // levels), and while HBM is plentiful straight to up to 4x the
            // need within a fifth of the free memory: each large hipMalloc
            // costs ~1 s per 50 GB, so a 1M-report sweep should grow its
            // slots a couple of times, not at every level
            size_t cap = std::max(nl, c->spare_cap + c->spare_cap / 4);
            size_t freeb = 0, totalb = 0;
            if (hipMemGetInfo(&freeb, &totalb) == hipSuccess) {
                const size_t per_node = 5 * S1 * 4;
                cap = std::max(cap, std::min(4 * nl, freeb / 5 / per_node));
            }
            // the spare may be a former slot that queued kernels still read:
            // retire it, and free the retired buffers first
            retire(c->fc_spare);
            c->spare_cap = 0;
            if (c->idle()) c->bury();
            ok = alloc(c->fc_spare, cap * 5 * S1 * 4);
            if (ok) c->spare_cap = cap;
        }
        if (!ok) {  // not enough HBM for the cache: evaluate without it
            lc->release();
            lc = nullptr;
            hit = false;
        } else {
            cin = hit ? lc->nd.as<uint32_t>() : nullptr;
            cout = c->fc_spare.as<uint32_t>();
        }
        if (!hit && lc) lc->drop();  // refilled by this call
    } else {
        c->lc[agg_id].drop();
    }
    // with the cache on, half of the free HBM: the other aggregator's slot may
    // still grow at this level
    const size_t per_report = wl.words * 4;
    // (an arena that already holds the whole batch needs no budget: skip the
    // free-memory query, ~tens of us per call)
    const bool fits = !c->budget && c->work.bytes / per_report >= round_up(n, 64) + pad;
    const uint64_t budget = fits ? (uint64_t)per_report * (round_up(n, 64) + pad)
                            : (lc && !c->budget) ? default_budget(c) * 2 / 3 : default_budget(c);
    // Plane rows are padded by stride_pad words: with a power-of-two row
    // length every word of a report sits at the same address bits modulo a
    // large power of two, and the 42-plane block loads of the binder sponges
    // all land on the same memory channels.
    size_t by_budget = (budget / per_report) / 64 * 64;
    if (by_budget > pad + 64) by_budget -= pad;  // the padded rows count against the budget too
    size_t chunk = std::min<size_t>(round_up(n, 64), by_budget);
    // The work buffer is an arena kept across calls: a call uses all of its
    // capacity (even past the budget: it is allocated already), and a new
    // one is at least c->work_arena bytes (within the budget), so a level
    // sweep whose trees grow from level to level does not re-allocate it at
    // every level.
    const size_t have = c->work.bytes / per_report;
    // An arena that holds half the batch in chunks of >= 64k reports is used
    // as it is (pipelined chunks of that size keep the GPU full and hide each
    // other's sponge tails) rather than re-allocated for a single chunk.
    const size_t need = std::min(chunk, round_up(n, 64)) + pad;
    if (have >= need || (2 * have >= need && have >= pad + 2 * 65536)) {
        chunk = std::min<size_t>(round_up(n, 64), (have - pad) / 64 * 64);
    } else {
        if (chunk < 64) return fail(c, MASTIC_ENOMEM, "work buffers of 64 reports exceed the memory budget");
        const size_t want = per_report * (chunk + pad);
        const size_t arena = std::max(want, std::min<size_t>(lc ? c->work_arena_fc : c->work_arena, budget));
        c->rk.valid = false;  // the arena may be re-allocated (possibly at the same address)
        if (!c->work.ensure(arena) && !c->work.ensure(want)) {
            // retired buffers (cache slots, evicted trees) are freed once the stream is idle
            if (c->graveyard.empty() || !c->idle())
                return fail(c, MASTIC_ENOMEM, "out of device memory (work %zu bytes)", want);
            c->bury();
            if (!c->work.ensure(arena) && !c->work.ensure(want))
                return fail(c, MASTIC_ENOMEM, "out of device memory (work %zu bytes)", want);
        }
        chunk = std::min<size_t>(round_up(n, 64), (c->work.bytes / per_report - pad) / 64 * 64);
    }
    if (c->budget) chunk = std::min(chunk, std::max<size_t>(by_budget, 64));  // an explicit budget caps chunks
    // MASTIC_CHUNK_REPORTS caps a chunk below what fits, so a large batch runs
    // as several pipelined chunks (the trailing sponges of one overlap the
    // evaluation of the next) instead of one chunk with an exposed tail
    const bool capped = c->chunk_max > 0 && round_up(c->chunk_max, 64) < chunk;
    if (capped) chunk = round_up(c->chunk_max, 64);
    // Several chunks: pipeline them through the two halves of the work arena
    // (chunk k+1 evaluates in one half while chunk k's last sponges, finalize
    // and copies run on the sponge stream over the other).
    const size_t half_cap = c->work.bytes / 2 / per_report;  // reports (padding rows included) per half
    const bool pipe = c->chunk_pipeline && n > chunk && chunk >= 128 && half_cap >= pad + 64;
    if (pipe) chunk = std::min(capped ? chunk : chunk / 2, half_cap - pad) / 64 * 64;
    const size_t half = c->work.bytes / 2 / 4 / 64 * 64;  // words: second half's offset
    const size_t nsev = 3 * (size_t)t->L + 12;          // sync events one chunk uses
    size_t evi = 0;
    hipEvent_t t0 = get_event(c, evi++), t1 = get_event(c, evi++);
    HIPCHK(c, hipEventRecord(t0, c->stream));
    hipEvent_t half_free[2] = {get_sync_event(c, 2 * nsev), get_sync_event(c, 2 * nsev + 1)};
    size_t k = 0;
    for (size_t b = 0; b < n; b += chunk, k++) {
        const int nn = (int)std::min(chunk, n - b);
        const int stride = (int)(round_up(nn, 64) + pad);
        const int h = pipe ? (int)(k & 1) : 0;
        if (pipe && k >= 2) HIPCHK(c, hipStreamWaitEvent(c->stream, half_free[h], 0));
        uint32_t* W = c->work.as<uint32_t>() + h * half;
        // pipelined chunks alternate between two sponge streams: a chunk's
        // sponges must not queue behind the previous chunk's trailing ones
        hipStream_t ss = (pipe && h) ? c->stream3 : c->stream2;
        hipStream_t tail = pipe ? ss : c->stream;
        rc = p.field == 64
                 ? run_chunk<F64>(c, rep, t, wl, agg_id, b, nn, stride, evi, lc, hit, cin, cout, W, ss, tail,
                                  h * nsev)
                 : run_chunk<F128>(c, rep, t, wl, agg_id, b, nn, stride, evi, lc, hit, cin, cout, W, ss, tail,
                                   h * nsev);
        if (rc) {
            if (lc) lc->drop();
            return rc;
        }
        if (pipe) HIPCHK(c, hipEventRecord(half_free[h], ss));
    }
    if (pipe) {
        // later work on the main stream (results, aggregate, the next call) sees every chunk's tail
        hipEvent_t done = get_sync_event(c, 2 * nsev + 2), done3 = get_sync_event(c, 2 * nsev + 3);
        HIPCHK(c, hipEventRecord(done, c->stream2));
        HIPCHK(c, hipEventRecord(done3, c->stream3));
        HIPCHK(c, hipStreamWaitEvent(c->stream, done, 0));
        HIPCHK(c, hipStreamWaitEvent(c->stream, done3, 0));
    }
    if (lc) {
        // the spare slot now holds this call's last level: it becomes the
        // aggregator's slot, and the old slot (read by this call's hit) the
        // spare, overwritten only by later calls' kernels (stream order)
        std::swap(lc->nd.p, c->fc_spare.p);
        std::swap(lc->nd.bytes, c->fc_spare.bytes);
        std::swap(lc->nodes_cap, c->spare_cap);
        lc->valid = true;
        lc->rep_id = rep->id;
        lc->rep_gen = rep->generation();
        lc->n = n;
        lc->key = lkey;
        lc->L = t->L;
        lc->n_parents.assign(t->n_parents.begin(), t->n_parents.begin() + t->L + 1);
        lc->paths.assign(t->child_path.begin() + t->off[t->L] * 8,
                         t->child_path.begin() + (t->off[t->L] + 2 * t->n_parents[t->L]) * 8);
    }
    c->last_hit = hit;
    HIPCHK(c, hipEventRecord(t1, c->stream));
    c->tm[c->tcur].n_eval = -(int)evi;  // timing pending (resolved by mastic_last_timing)
    R.ready = true;
    return 0;
}

// Report-major wire rows of plane segments into dst (device), on c->stream.
static int gather_rows(mastic_ctx* c, const RowSegs& sg, size_t n, size_t stride, void* dst) {
    const size_t words = (size_t)sg.words[0] + sg.words[1] + sg.words[2];
    if (n == 0 || words == 0) return 0;
    const size_t total = n * words;
    // grid-stride kernel: at most 2^20 workgroups (2^28 work-items) per launch
    const size_t blocks = std::min<size_t>((total + 255) / 256, (size_t)1 << 20);
    hipLaunchKernelGGL(k_gather_rows, dim3((unsigned)blocks), dim3(256), 0, c->stream, sg, (int)n, (int)stride,
                       (uint32_t*)dst);
    HIPCHK(c, hipGetLastError());
    return 0;
}

// The prep shares of result slot R as wire rows (mastic.py:543-552):
// eval_proof || [jr_part] || [verifier].
static RowSegs prep_share_segs(const McParams& p, const Result& R) {
    RowSegs sg{};
    sg.seg[0] = R.eval_proof.as<uint32_t>();
    sg.words[0] = 8;
    if (R.weight_check) {
        int k = 1;
        if (p.joint_rand_len > 0) {
            sg.seg[k] = R.jr_part.as<uint32_t>();
            sg.words[k++] = 8;
        }
        sg.seg[k] = R.verifier.as<uint32_t>();
        sg.words[k] = p.verifier_len * p.w32;
    }
    return sg;
}

extern "C" int mastic_prep_result(mastic_ctx* c, int agg_id, uint8_t* prep_shares, uint8_t* jr_seeds,
                                  uint8_t* out_shares, int32_t* status) {
    DeviceScope ds_(c);
    if (!c || (agg_id != 0 && agg_id != 1)) return fail(c, MASTIC_EINVAL, "invalid aggregator ID");
    Result& R = c->res[agg_id];
    if (!R.ready) return fail(c, MASTIC_EINVAL, "no prep_init result for this aggregator");
    c->tcur = agg_id;
    const McParams& p = c->p;
    const size_t n = R.n, S = R.stride;
    // Every output is encoded on the GPU into a staging buffer (planes ->
    // report-major wire bytes) and copied out once: no per-report host loop.
    auto emit = [&](const RowSegs& sg, void* host) -> int {
        const size_t bytes = n * 4 * ((size_t)sg.words[0] + sg.words[1] + sg.words[2]);
        if (!host || bytes == 0) return 0;
        if (!c->stage.grow(bytes)) return fail(c, MASTIC_ENOMEM, "out of device memory (result staging)");
        if (gather_rows(c, sg, n, S, c->stage.p)) return -1;
        HIPCHK(c, hipMemcpyAsync(host, c->stage.p, bytes, hipMemcpyDeviceToHost, c->stream));
        HIPCHK(c, hipStreamSynchronize(c->stream));
        return 0;
    };
    HIPCHK(c, hipStreamSynchronize(c->stream));
    c->bury();  // the stream is idle (it joined the sponge stream before k_finalize)
    if (n == 0) return 0;
    if (emit(prep_share_segs(p, R), prep_shares)) return -1;
    if (jr_seeds && !(R.weight_check && p.joint_rand_len > 0)) {
        memset(jr_seeds, 0, 32 * n);  // no joint rand in this call
    } else if (emit(RowSegs{{R.jr_seed.as<uint32_t>(), nullptr, nullptr}, {8, 0, 0}}, jr_seeds)) {
        return -1;
    }
    const int ow = R.n_prefixes * (1 + p.output_len) * p.w32;
    if (emit(RowSegs{{R.out.as<uint32_t>(), nullptr, nullptr}, {ow, 0, 0}}, out_shares)) return -1;
    if (emit(RowSegs{{(const uint32_t*)R.status.p, nullptr, nullptr}, {1, 0, 0}}, status)) return -1;
    return 0;
}

extern "C" int mastic_decide_results(mastic_ctx* c, const uint8_t* app_ctx, size_t ctx_len, uint8_t* accept_out,
                                     uint8_t* decide_out) {
    DeviceScope ds_(c);
    if (!c) return MASTIC_EINVAL;
    Result &R0 = c->res[0], &R1 = c->res[1];
    if (!R0.ready || !R1.ready) return fail(c, MASTIC_EINVAL, "decide needs both aggregators' prep_init results");
    if (R0.n != R1.n || R0.weight_check != R1.weight_check || R0.n_prefixes != R1.n_prefixes)
        return fail(c, MASTIC_EINVAL, "the two prep_init results are for different batches / agg params");
    const size_t n = R0.n, S = R0.stride;
    if (n == 0) return 0;
    int rc = build_prefixes(c, app_ctx, ctx_len, nullptr, 0);
    if (rc) return rc;
    const McParams& p = c->p;
    const size_t psz = mc_prep_share_size(p, R0.weight_check);
    // both prep shares as wire rows (k_decide's input), decide, accept
    const size_t need = 2 * n * psz + 32 * n + 2 * n + 256 + S * 4 * (size_t)std::max(1, p.verifier_len * p.w32);
    if (!c->stage.grow(need)) return fail(c, MASTIC_ENOMEM, "out of device memory (decide staging)");
    uint8_t* ps0 = c->stage.as<uint8_t>();
    uint8_t* ps1 = ps0 + n * psz;
    uint8_t* msg = ps1 + n * psz;
    uint8_t* code = msg + 32 * n;
    uint8_t* acc = code + n;
    uint32_t* ver = (uint32_t*)(((uintptr_t)(acc + n) + 255) & ~(uintptr_t)255);  // FLP scratch planes
    if (gather_rows(c, prep_share_segs(p, R0), n, S, ps0)) return -1;
    if (gather_rows(c, prep_share_segs(p, R1), n, S, ps1)) return -1;
    HIPCHK(c, hipMemsetAsync(msg, 0, 32 * n, c->stream));
    const dim3 grid((unsigned)((n + 255) / 256));
    if (p.field == 64)
        hipLaunchKernelGGL(k_decide<F64>, grid, dim3(256), 0, c->stream, p, (int)n, (int)S, R0.weight_check, ps0, ps1,
                           (int)psz, ver, (const PrefixState*)c->pfx.p, msg, code);
    else
        hipLaunchKernelGGL(k_decide<F128>, grid, dim3(256), 0, c->stream, p, (int)n, (int)S, R0.weight_check, ps0,
                           ps1, (int)psz, ver, (const PrefixState*)c->pfx.p, msg, code);
    HIPCHK(c, hipGetLastError());
    hipLaunchKernelGGL(k_accept, grid, dim3(256), 0, c->stream, (int)n, (int)S,
                       (int)(R0.weight_check && p.joint_rand_len > 0), code, (const int32_t*)R0.status.p,
                       (const int32_t*)R1.status.p, msg, R0.jr_seed.as<uint32_t>(), R1.jr_seed.as<uint32_t>(), acc);
    HIPCHK(c, hipGetLastError());
    if (accept_out) HIPCHK(c, hipMemcpyAsync(accept_out, acc, n, hipMemcpyDeviceToHost, c->stream));
    if (decide_out) HIPCHK(c, hipMemcpyAsync(decide_out, code, n, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    c->bury();
    return 0;
}

// Fold of the out shares of the last prep_init of agg_id into dagg (device).
static int aggregate_impl(mastic_ctx* c, int agg_id, const uint8_t* valid, uint32_t* dagg) {
    Result& R = c->res[agg_id];
    const McParams& p = c->p;
    const size_t rows = (size_t)R.n_prefixes * (1 + p.output_len);
    const uint8_t* dv = nullptr;
    if (valid && R.n) {
        if (!c->agg_valid.grow(R.n)) return fail(c, MASTIC_ENOMEM, "out of device memory");
        HIPCHK(c, hipMemcpyAsync(c->agg_valid.p, valid, R.n, hipMemcpyHostToDevice, c->stream));
        dv = c->agg_valid.as<uint8_t>();
    }
    if (!rows) return 0;
    // few rows over many reports (a sweep level: ~700 rows x 1M reports):
    // split the reports into chunks so the grid fills the chip, then merge
    // the chunks' partial sums mod p (k_fold_shares)
    const size_t target = (size_t)c->n_cus * 16;
    size_t chunks = 1;
    if (rows < target && R.n >= 8192)
        chunks = std::min<size_t>({(target + rows - 1) / rows, R.n / 4096, (size_t)1024});
    // (an empty batch still writes its all-zero agg share: one chunk)
    const size_t chunk = chunks > 1 ? round_up((R.n + chunks - 1) / chunks, 256) : std::max<size_t>(R.n, 1);
    chunks = std::max<size_t>(1, (R.n + chunk - 1) / chunk);
    uint32_t* dst = dagg;
    if (chunks > 1) {
        if (!c->agg_part.ensure(std::max<size_t>(chunks * rows * p.w32 * 4, (size_t)1 << 20)))
            return fail(c, MASTIC_ENOMEM, "out of device memory");
        dst = c->agg_part.as<uint32_t>();
    }
    const dim3 grid((unsigned)rows, (unsigned)chunks);
    if (p.field == 64)
        hipLaunchKernelGGL(k_fold<F64>, grid, dim3(256), 0, c->stream, R.out.as<uint32_t>(), (int)R.n, (int)R.stride,
                           dv, (int)chunk, dst);
    else
        hipLaunchKernelGGL(k_fold<F128>, grid, dim3(256), 0, c->stream, R.out.as<uint32_t>(), (int)R.n, (int)R.stride,
                           dv, (int)chunk, dst);
    HIPCHK(c, hipGetLastError());
    if (chunks > 1) {
        const dim3 g2((unsigned)((rows + 255) / 256));
        if (p.field == 64)
            hipLaunchKernelGGL(k_fold_shares<F64>, g2, dim3(256), 0, c->stream, (const uint32_t*)dst, (int)chunks,
                               (int)rows, dagg);
        else
            hipLaunchKernelGGL(k_fold_shares<F128>, g2, dim3(256), 0, c->stream, (const uint32_t*)dst, (int)chunks,
                               (int)rows, dagg);
        HIPCHK(c, hipGetLastError());
    }
    return 0;
}

extern "C" int mastic_aggregate(mastic_ctx* c, int agg_id, const uint8_t* valid, uint8_t* agg_share) {
    DeviceScope ds_(c);
    if (!c || (agg_id != 0 && agg_id != 1)) return fail(c, MASTIC_EINVAL, "invalid aggregator ID");
    Result& R = c->res[agg_id];
    if (!R.ready) return fail(c, MASTIC_EINVAL, "no prep_init result for this aggregator");
    const McParams& p = c->p;
    const size_t rows = (size_t)R.n_prefixes * (1 + p.output_len);
    if (!c->agg_out.grow(std::max<size_t>(rows, 1) * p.w32 * 4)) return fail(c, MASTIC_ENOMEM, "out of device memory");
    int rc = aggregate_impl(c, agg_id, valid, c->agg_out.as<uint32_t>());
    if (rc) return rc;
    if (agg_share && rows)
        HIPCHK(c, hipMemcpyAsync(agg_share, c->agg_out.p, rows * p.w32 * 4, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    return 0;
}

// (ABI 6: the only name of this function; mastic_aggregate_device, whose
// argument count changed between ABI 3, 4 and 5, is gone)
extern "C" int mastic_aggregate_device_on_stream(mastic_ctx* c, int agg_id, const uint8_t* valid,
                                                 void* dev_agg_share, void* caller_stream) {
    DeviceScope ds_(c);
    if (!c || (agg_id != 0 && agg_id != 1)) return fail(c, MASTIC_EINVAL, "invalid aggregator ID");
    Result& R = c->res[agg_id];
    if (!R.ready) return fail(c, MASTIC_EINVAL, "no prep_init result for this aggregator");
    const size_t rows = (size_t)R.n_prefixes * (1 + c->p.output_len);
    if (rows && !dev_agg_share) return fail(c, MASTIC_EINVAL, "null agg share buffer");
    // the buffer may have been allocated / filled by work queued on the
    // caller's stream (e.g. a torch allocation's fill): the fold writes it
    // only after that work, ordered by an event (no device-wide sync)
    if (!c->fold_ev) HIPCHK(c, hipEventCreateWithFlags(&c->fold_ev, hipEventDisableTiming));
    HIPCHK(c, hipEventRecord(c->fold_ev, (hipStream_t)caller_stream));
    HIPCHK(c, hipStreamWaitEvent(c->stream, c->fold_ev, 0));
    int rc = aggregate_impl(c, agg_id, valid, (uint32_t*)dev_agg_share);
    if (rc) return rc;
    HIPCHK(c, hipStreamSynchronize(c->stream));  // the caller's stream (e.g. RCCL's) reads it next
    return 0;
}

extern "C" int mastic_fold_shares(mastic_ctx* c, const void* dev_shares, size_t n_shares, size_t n_elems,
                                  void* dev_out, void* producer_stream) {
    DeviceScope ds_(c);
    if (!c || (!dev_shares && n_shares) || !dev_out) return MASTIC_EINVAL;
    if (n_elems == 0) return 0;
    // the shares were written on the caller's stream (e.g. an RCCL all-gather):
    // order the fold after that stream's work with an event, not a device sync
    if (!c->fold_ev) HIPCHK(c, hipEventCreateWithFlags(&c->fold_ev, hipEventDisableTiming));
    HIPCHK(c, hipEventRecord(c->fold_ev, (hipStream_t)producer_stream));
    HIPCHK(c, hipStreamWaitEvent(c->stream, c->fold_ev, 0));
    const dim3 grid((unsigned)((n_elems + 255) / 256));
    if (c->p.field == 64)
        hipLaunchKernelGGL(k_fold_shares<F64>, grid, dim3(256), 0, c->stream, (const uint32_t*)dev_shares,
                           (int)n_shares, (int)n_elems, (uint32_t*)dev_out);
    else
        hipLaunchKernelGGL(k_fold_shares<F128>, grid, dim3(256), 0, c->stream, (const uint32_t*)dev_shares,
                           (int)n_shares, (int)n_elems, (uint32_t*)dev_out);
    HIPCHK(c, hipGetLastError());
    HIPCHK(c, hipStreamSynchronize(c->stream));
    return 0;
}

// ---- multi-GPU merge over the ctx's own RCCL communicator --
//
// Failure model.  Every collective entry point (mastic_allgather_fold,
// mastic_merge_host, mastic_aggregate_merged) first does all of its
// rank-local work -- argument checks, staging allocations, the local fold --
// and then joins an agreement round: one 32-byte CommStatus per rank (its
// error code, the entry point, n_local, n_elems), all-gathered into buffers
// sized at mastic_comm_init.  A rank whose local work failed still joins it,
// so no peer is left waiting inside a data all-gather: a rank that failed
// returns its own error, every other rank the code of the lowest failing
// rank, and ranks whose calls disagree on the entry point or the share
// geometry all return MASTIC_EINVAL, before any share bytes move.  Only when
// every rank is ready do the data all-gather and the GF(p) fold run.  Every
// wait on the communicator is bounded by the ctx's timeout
// (mastic_comm_init_timeout): a peer that never joins (it crashed, or is stuck
// elsewhere) becomes MASTIC_ETIMEDOUT.  An init that times out is abandoned
// (its thread keeps it; the ctx stays world 1); a collective that times out
// aborts the communicator (ncclCommAbort), and later collective calls then
// fail with MASTIC_EHIP -- never a silent world-1 merge -- until
// mastic_comm_destroy and a new mastic_comm_init.

namespace {
// RCCL is bound on first use of a communicator entry point (dlopen), so a
// single-GPU user of the library has no load-time dependency on librccl; a
// process that already holds it (e.g. PyTorch's copy) shares that one.
struct RcclApi {
    bool ok = false;
    std::string why;
    decltype(&ncclGetUniqueId) GetUniqueId = nullptr;
    decltype(&ncclCommInitRank) CommInitRank = nullptr;
    decltype(&ncclCommGetAsyncError) CommGetAsyncError = nullptr;
    decltype(&ncclCommAbort) CommAbort = nullptr;
    decltype(&ncclCommFinalize) CommFinalize = nullptr;
    decltype(&ncclCommDestroy) CommDestroy = nullptr;
    decltype(&ncclAllGather) AllGather = nullptr;
    decltype(&ncclGetErrorString) GetErrorString = nullptr;
};

const RcclApi& rccl() {
    static const RcclApi api = [] {
        RcclApi a;
        void* h = nullptr;
        // test hook: MASTIC_RCCL_LIB names the library to bind instead (the
        // shared-memory stand-in of tests/host/fake_rccl.cpp, which lets several
        // processes on one GPU form a communicator); no fallback to RCCL
        const char* hook = getenv("MASTIC_RCCL_LIB");
        if (hook && *hook) {
            h = dlopen(hook, RTLD_NOW | RTLD_LOCAL);
        } else {
            for (const char* name : {"librccl.so.1", "/opt/rocm/lib/librccl.so.1", "librccl.so"})
                if ((h = dlopen(name, RTLD_NOW | RTLD_LOCAL))) break;
        }
        if (!h) {
            const char* e = dlerror();
            a.why = e ? e : "librccl.so.1 not found";
            return a;
        }
        bool all = true;
        auto bind = [&](auto& fn, const char* name) {
            fn = reinterpret_cast<std::remove_reference_t<decltype(fn)>>(dlsym(h, name));
            if (!fn && all) a.why = std::string("librccl lacks ") + name;
            all = all && fn;
        };
        bind(a.GetUniqueId, "ncclGetUniqueId");
        bind(a.CommInitRank, "ncclCommInitRank");
        bind(a.CommGetAsyncError, "ncclCommGetAsyncError");
        bind(a.CommAbort, "ncclCommAbort");
        bind(a.CommFinalize, "ncclCommFinalize");
        bind(a.CommDestroy, "ncclCommDestroy");
        bind(a.AllGather, "ncclAllGather");
        bind(a.GetErrorString, "ncclGetErrorString");
        a.ok = all;
        return a;
    }();
    return api;
}

// One communicator init on its own thread (mastic_comm_init_timeout).
struct CommInitJob {
    std::mutex mu;
    std::condition_variable cv;
    bool done = false, abandoned = false;
    ncclComm_t comm = nullptr;
    ncclResult_t r = ncclSuccess;
    hipError_t dev_err = hipSuccess;
};
}  // namespace

// ctx teardown: its queued work is waited for, then the communicator is
// released locally (ncclCommAbort never waits on peers that may be gone).
void mastic_ctx::comm_release() {
    (void)hipStreamSynchronize(stream);
    (void)rccl().CommAbort(comm);
    comm = nullptr;
}

// Abort the ctx's communicator after a failed or timed-out RCCL step: its
// kernels see the abort flag and exit, the ctx keeps comm_broken so later
// collective calls fail instead of silently folding as world 1.
// MASTIC_TRACE_COMM: mark step i of the agreement round on the ctx's stream;
// a timed-out wait reports which marks the stream has passed.
static void comm_mark(mastic_ctx* c, int i) {
    if (!trace_comm()) return;
    if (!c->comm_marks[i] && hipEventCreateWithFlags(&c->comm_marks[i], hipEventDisableTiming) != hipSuccess) return;
    (void)hipEventRecord(c->comm_marks[i], c->stream);
}
static void comm_marks_report(mastic_ctx* c) {
    if (!trace_comm()) return;
    for (int i = 0; i < 3; i++)
        if (c->comm_marks[i])
            fprintf(stderr, "[mastic comm]   mark %d (%s): %s\n", i,
                    (const char*[]){"status uploaded", "status all-gather queued", "status download queued"}[i],
                    hipEventQuery(c->comm_marks[i]) == hipSuccess ? "passed" : "not passed");
}

static int comm_abort(mastic_ctx* c, int code, const char* fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    if (trace_comm()) fprintf(stderr, "[mastic comm] abort: %s\n", buf);
    if (c->comm) {
        const ncclResult_t r = rccl().CommAbort(c->comm);
        if (trace_comm()) fprintf(stderr, "[mastic comm] ncclCommAbort -> %d\n", (int)r);
    }
    c->comm = nullptr;
    c->comm_broken = true;
    return fail(c, code, "%s; the communicator was aborted", buf);
}

// The result of an RCCL call on the ctx's communicator; a call that reports
// ncclInProgress (a non-blocking communicator's) is polled until it settles,
// within the ctx's timeout.
static int comm_settle(mastic_ctx* c, ncclResult_t r, const char* what) {
    const double t0 = now_ms();
    while (r == ncclInProgress) {
        if (now_ms() - t0 > c->comm_timeout_ms)
            return comm_abort(c, MASTIC_ETIMEDOUT, "RCCL %s did not complete within %d ms", what, c->comm_timeout_ms);
        std::this_thread::yield();
        ncclResult_t st = ncclSuccess;
        const ncclResult_t q = rccl().CommGetAsyncError(c->comm, &st);
        r = q != ncclSuccess ? q : st;
    }
    if (r != ncclSuccess) return comm_abort(c, MASTIC_EHIP, "RCCL %s: %s", what, rccl().GetErrorString(r));
    return 0;
}

// Wait for c->stream, which carries an RCCL collective: bounded by the ctx's
// timeout (a peer that never joins), watching the communicator's own errors.
static int comm_wait(mastic_ctx* c, const char* what) {
    const double t0 = now_ms();
    for (int spin = 0;; spin++) {
        const hipError_t e = hipStreamQuery(c->stream);
        if (e == hipSuccess) return 0;
        if (e != hipErrorNotReady) {
            (void)hipGetLastError();
            return comm_abort(c, MASTIC_EHIP, "%s: %s", what, hipGetErrorString(e));
        }
        ncclResult_t st = ncclSuccess;
        if (rccl().CommGetAsyncError(c->comm, &st) == ncclSuccess && st != ncclSuccess && st != ncclInProgress)
            return comm_abort(c, MASTIC_EHIP, "RCCL %s: %s", what, rccl().GetErrorString(st));
        if (now_ms() - t0 > c->comm_timeout_ms) {
            comm_marks_report(c);
            return comm_abort(c, MASTIC_ETIMEDOUT, "%s: a peer rank did not join within %d ms", what,
                              c->comm_timeout_ms);
        }
        if (spin < 2000)
            std::this_thread::yield();
        else
            std::this_thread::sleep_for(std::chrono::microseconds(50));
    }
}

// A staging buffer of a collective call (counts against the fail_allocs
// test hook when it must actually allocate).
static bool comm_grow(mastic_ctx* c, DevBuf& b, size_t want) {
    if (want <= b.bytes && b.p) return true;
    if (c->inject_alloc_failure()) return false;
    return b.grow(want);
}

// The agreement round (see the failure model above).  local_rc: the outcome
// of this rank's local work (0, or a code whose text is already in c->err).
// Returns 0 iff every rank is ready for the data exchange.
static int comm_agree(mastic_ctx* c, int local_rc, uint32_t op, size_t n_local, size_t n_elems) {
    if (!c->comm) {
        if (c->comm_broken && !local_rc)
            return fail(c, MASTIC_EHIP, "the ctx's communicator was aborted after an earlier failure "
                                        "(mastic_comm_destroy, then mastic_comm_init)");
        return local_rc;  // world 1
    }
    // this rank's queued work (its prep_init, the local fold) first, unbounded:
    // the timeout below then measures only the wait for the peers
    {
        const hipError_t e = hipStreamSynchronize(c->stream);
        if (e != hipSuccess && !local_rc) {
            (void)hipGetLastError();
            local_rc = fail(c, MASTIC_EHIP, "%s: local work failed: %s", comm_op_name(op), hipGetErrorString(e));
        }
    }
    const std::string local_err = c->err;
    CommStatus* h = (CommStatus*)c->comm_st_host;  // [0]: this rank's record, [1 + r]: rank r's
    h[0] = CommStatus{local_rc, op, (uint64_t)n_local, (uint64_t)n_elems, COMM_MAGIC, 0};
    uint8_t* d = c->comm_st.as<uint8_t>();
    hipError_t e = hipMemcpyAsync(d, h, sizeof(CommStatus), hipMemcpyHostToDevice, c->stream);
    if (e != hipSuccess) {
        (void)hipGetLastError();
        return comm_abort(c, local_rc ? local_rc : MASTIC_EHIP, "%s: status upload: %s", comm_op_name(op),
                          hipGetErrorString(e));
    }
    comm_mark(c, 0);
    int rc = comm_settle(c, rccl().AllGather(d, d + sizeof(CommStatus), sizeof(CommStatus), ncclUint8, c->comm,
                                             c->stream), "status all-gather");
    if (rc) return local_rc ? local_rc : rc;
    comm_mark(c, 1);
    e = hipMemcpyAsync(h + 1, d + sizeof(CommStatus), sizeof(CommStatus) * (size_t)c->comm_n, hipMemcpyDeviceToHost,
                       c->stream);
    if (e != hipSuccess) {
        (void)hipGetLastError();
        return comm_abort(c, local_rc ? local_rc : MASTIC_EHIP, "%s: status download: %s", comm_op_name(op),
                          hipGetErrorString(e));
    }
    comm_mark(c, 2);
    rc = comm_wait(c, "status all-gather");
    if (rc) return local_rc ? local_rc : rc;
    const CommVerdict v = comm_decide(h + 1, c->comm_n, op, n_local, n_elems);
    const int rc_all = comm_rank_result(v, local_rc, MASTIC_EINVAL);
    if (local_rc) {
        c->err = local_err;
        return local_rc;
    }
    if (v.first_bad >= 0)
        return fail(c, rc_all, "%s failed on rank %d (code %d); no shares were exchanged", comm_op_name(op),
                    v.first_bad, v.bad_rc);
    if (v.mismatch >= 0) {
        const int mismatch = v.mismatch;
        const CommStatus& s = h[1 + mismatch];
        return fail(c, MASTIC_EINVAL,
                    "ranks disagree on the collective call: rank %d called %s with %llu x %llu elements, this rank "
                    "%s with %zu x %zu; no shares were exchanged",
                    mismatch, comm_op_name(s.op), (unsigned long long)s.n_local, (unsigned long long)s.n_elems,
                    comm_op_name(op), n_local, n_elems);
    }
    return 0;
}

// Staging for the data all-gather of n_local shares of n_elems elements from
// every rank (allocated in the local phase, before the agreement).
static bool comm_stage_gather(mastic_ctx* c, size_t n_local, size_t n_elems) {
    return !c->comm || comm_grow(c, c->comm_gather, std::max<size_t>(n_local * n_elems * c->p.w32 * 4, 4) * c->comm_n);
}

// dev_out = sum mod p of the n_local shares of every rank (n_elems elements
// each), queued on c->stream after a successful agreement: one ncclAllGather
// of this rank's shares into the rank-ordered comm_gather, then
// k_fold_shares over the n_local x nranks shares (RCCL's integer sum is not
// GF(p) addition).  Without a communicator the local shares are folded
// directly (world 1).
static int allgather_fold_impl(mastic_ctx* c, const uint32_t* local, size_t n_local, size_t n_elems, uint32_t* out) {
    const size_t local_bytes = n_local * n_elems * c->p.w32 * 4;
    const uint32_t* src = local;
    size_t n_shares = n_local;
    if (c->comm && local_bytes) {
        int rc = comm_settle(c, rccl().AllGather(local, c->comm_gather.p, local_bytes, ncclUint8, c->comm, c->stream),
                             "share all-gather");
        if (rc) return rc;
        src = c->comm_gather.as<uint32_t>();
        n_shares = n_local * (size_t)c->comm_n;
    }
    const dim3 grid((unsigned)((n_elems + 255) / 256));
    if (c->p.field == 64)
        hipLaunchKernelGGL(k_fold_shares<F64>, grid, dim3(256), 0, c->stream, src, (int)n_shares, (int)n_elems, out);
    else
        hipLaunchKernelGGL(k_fold_shares<F128>, grid, dim3(256), 0, c->stream, src, (int)n_shares, (int)n_elems, out);
    HIPCHK(c, hipGetLastError());
    return 0;
}

// The end of a collective call: its queued work (the data all-gather, the
// fold, the copy out) done, bounded by the timeout when RCCL is in it.
static int comm_finish(mastic_ctx* c, uint32_t op) {
    if (c->comm) return comm_wait(c, comm_op_name(op));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    return 0;
}

// The merged share to the caller's host buffer, AFTER comm_finish: a copy to
// pageable memory is synchronous, so queued behind a data all-gather that a
// dead peer never completes it would block this thread past every bound
// (found by tests/test_gpu_comm_nrank.py: a peer lost between the agreement
// round and the data all-gather).
static int comm_copy_out(mastic_ctx* c, void* host_out, size_t bytes) {
    HIPCHK(c, hipMemcpyAsync(host_out, c->comm_out.p, bytes, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    return 0;
}

// Shape limits of the fold kernel (k_fold_shares takes int counts).
static int comm_check_counts(mastic_ctx* c, size_t n_local, size_t n_elems) {
    if (n_local * (size_t)c->comm_n > (size_t)INT32_MAX || n_elems > (size_t)INT32_MAX)
        return fail(c, MASTIC_EINVAL, "too many shares to fold");
    return 0;
}

extern "C" int mastic_comm_unique_id(uint8_t id_out[MASTIC_COMM_ID_BYTES]) {
    static_assert(sizeof(ncclUniqueId) == MASTIC_COMM_ID_BYTES, "ncclUniqueId size");
    if (!id_out) return MASTIC_EINVAL;
    if (!rccl().ok) return MASTIC_ENODEV;
    ncclUniqueId id;
    if (rccl().GetUniqueId(&id) != ncclSuccess) return MASTIC_EHIP;
    std::memcpy(id_out, &id, sizeof(id));
    return 0;
}

extern "C" int mastic_comm_init_timeout(mastic_ctx* c, int nranks, int rank, const uint8_t id[MASTIC_COMM_ID_BYTES],
                                        int timeout_ms) {
    DeviceScope ds_(c);
    if (!c) return MASTIC_EINVAL;
    if (!id || nranks < 1 || rank < 0 || rank >= nranks) return fail(c, MASTIC_EINVAL, "invalid communicator rank");
    if (c->comm) return fail(c, MASTIC_EINVAL, "the ctx already has a communicator");
    if (!rccl().ok) return fail(c, MASTIC_ENODEV, "RCCL is not available: %s", rccl().why.c_str());
    c->comm_timeout_ms = timeout_ms > 0 ? timeout_ms : MASTIC_COMM_TIMEOUT_MS;
    // the agreement round's buffers, before joining: a rank that cannot
    // allocate them fails here, before any collective
    const size_t st_bytes = sizeof(CommStatus) * ((size_t)nranks + 1);
    if (!c->comm_st.ensure(st_bytes)) return fail(c, MASTIC_ENOMEM, "out of device memory");
    if (c->comm_st_host_n < (size_t)nranks + 1) {
        if (c->comm_st_host) (void)hipHostFree(c->comm_st_host);
        c->comm_st_host = nullptr;
        c->comm_st_host_n = 0;
        HIPCHK(c, hipHostMalloc(&c->comm_st_host, st_bytes, hipHostMallocDefault));
        c->comm_st_host_n = (size_t)nranks + 1;
    }
    ncclUniqueId uid;
    std::memcpy(&uid, id, sizeof(uid));
    // RCCL's init blocks until every rank has joined -- in its bootstrap,
    // even for a communicator configured non-blocking (measured on RCCL
    // 2.27.7: ncclCommInitRankConfig with blocking = 0 did not return while
    // a peer was missing) -- so it runs on a thread of its own and this call
    // waits for it with the ctx's bound.  An init the caller gave up on stays
    // with its thread, which releases the communicator (ncclCommAbort) if the
    // peers ever arrive; the ctx stays world 1.
    auto job = std::make_shared<CommInitJob>();
    const int dev = c->device;
    try {
        std::thread([job, nranks, uid, rank, dev] {
            ncclComm_t comm = nullptr;
            ncclResult_t r = ncclSystemError;
            const hipError_t e = hipSetDevice(dev);
            if (e == hipSuccess) r = rccl().CommInitRank(&comm, nranks, uid, rank);
            std::unique_lock<std::mutex> lk(job->mu);
            job->comm = comm;
            job->r = r;
            job->dev_err = e;
            job->done = true;
            const bool given_up = job->abandoned;
            lk.unlock();
            job->cv.notify_all();
            if (given_up && comm) (void)rccl().CommAbort(comm);
        }).detach();
    } catch (const std::system_error&) {
        return fail(c, MASTIC_EHIP, "cannot start the RCCL init thread");
    }
    std::unique_lock<std::mutex> lk(job->mu);
    if (!job->cv.wait_for(lk, std::chrono::milliseconds(c->comm_timeout_ms), [&] { return job->done; })) {
        job->abandoned = true;
        if (trace_comm()) fprintf(stderr, "[mastic comm] init of rank %d of %d timed out\n", rank, nranks);
        return fail(c, MASTIC_ETIMEDOUT,
                    "RCCL init: not every rank joined within %d ms (the pending init is abandoned; the ctx stays "
                    "world 1)", c->comm_timeout_ms);
    }
    if (trace_comm()) fprintf(stderr, "[mastic comm] ncclCommInitRank(%d of %d) -> %d\n", rank, nranks, (int)job->r);
    if (job->dev_err != hipSuccess) return fail(c, MASTIC_EHIP, "hipSetDevice: %s", hipGetErrorString(job->dev_err));
    if (job->r != ncclSuccess) {
        if (job->comm) (void)rccl().CommAbort(job->comm);
        return fail(c, MASTIC_EHIP, "RCCL init: %s", rccl().GetErrorString(job->r));
    }
    c->comm = job->comm;
    c->comm_n = nranks;
    c->comm_rank = rank;
    c->comm_broken = false;
    return 0;
}

extern "C" int mastic_comm_init(mastic_ctx* c, int nranks, int rank, const uint8_t id[MASTIC_COMM_ID_BYTES]) {
    return mastic_comm_init_timeout(c, nranks, rank, id, MASTIC_COMM_TIMEOUT_MS);
}

extern "C" int mastic_comm_info(const mastic_ctx* c, int* nranks, int* rank) {
    if (!c) return MASTIC_EINVAL;
    if (nranks) *nranks = c->comm_n;
    if (rank) *rank = c->comm_rank;
    return 0;
}

extern "C" int mastic_comm_destroy(mastic_ctx* c) {
    DeviceScope ds_(c);
    if (!c) return MASTIC_EINVAL;
    int rc = 0;
    if (c->comm) {
        rc = comm_wait(c, "mastic_comm_destroy");
        if (!rc) rc = comm_settle(c, rccl().CommFinalize(c->comm), "finalize");
        if (!rc) {
            const ncclResult_t r = rccl().CommDestroy(c->comm);
            if (r != ncclSuccess) rc = fail(c, MASTIC_EHIP, "RCCL destroy: %s", rccl().GetErrorString(r));
        }
    }
    c->comm = nullptr;
    c->comm_n = 1;
    c->comm_rank = 0;
    c->comm_broken = false;
    return rc;
}

extern "C" int mastic_allgather_fold(mastic_ctx* c, const void* dev_local, size_t n_local, size_t n_elems,
                                     void* dev_out, void* caller_stream) {
    DeviceScope ds_(c);
    if (!c) return MASTIC_EINVAL;
    int rc = 0;
    if (n_elems && (!dev_out || (n_local && !dev_local))) rc = fail(c, MASTIC_EINVAL, "null share buffer");
    if (!rc) rc = comm_check_counts(c, n_local, n_elems);
    if (!rc && n_elems && !comm_stage_gather(c, n_local, n_elems)) rc = fail(c, MASTIC_ENOMEM, "out of device memory");
    if (!rc && n_elems) {
        if (!c->fold_ev && hipEventCreateWithFlags(&c->fold_ev, hipEventDisableTiming) != hipSuccess)
            rc = fail(c, MASTIC_EHIP, "hipEventCreateWithFlags failed");
        if (!rc && (hipEventRecord(c->fold_ev, (hipStream_t)caller_stream) != hipSuccess ||
                    hipStreamWaitEvent(c->stream, c->fold_ev, 0) != hipSuccess))
            rc = fail(c, MASTIC_EHIP, "ordering after the caller's stream failed");
    }
    rc = comm_agree(c, rc, COMM_ALLGATHER_FOLD, n_local, n_elems);
    if (rc || n_elems == 0) return rc;
    rc = allgather_fold_impl(c, (const uint32_t*)dev_local, n_local, n_elems, (uint32_t*)dev_out);
    if (rc) return rc;
    return comm_finish(c, COMM_ALLGATHER_FOLD);
}

extern "C" int mastic_merge_host(mastic_ctx* c, const uint8_t* host_local, size_t n_local, size_t n_elems,
                                 uint8_t* host_out) {
    DeviceScope ds_(c);
    if (!c) return MASTIC_EINVAL;
    const size_t ebytes = (size_t)c->p.w32 * 4;
    int rc = 0;
    if (n_elems && (!host_out || (n_local && !host_local))) rc = fail(c, MASTIC_EINVAL, "null share buffer");
    if (!rc) rc = comm_check_counts(c, n_local, n_elems);
    if (!rc && n_elems &&
        (!comm_grow(c, c->comm_local, std::max<size_t>(n_local, 1) * n_elems * ebytes) ||
         !comm_grow(c, c->comm_out, n_elems * ebytes) || !comm_stage_gather(c, n_local, n_elems)))
        rc = fail(c, MASTIC_ENOMEM, "out of device memory");
    if (!rc && n_elems && n_local &&
        hipMemcpyAsync(c->comm_local.p, host_local, n_local * n_elems * ebytes, hipMemcpyHostToDevice, c->stream) !=
            hipSuccess)
        rc = fail(c, MASTIC_EHIP, "share upload failed");
    rc = comm_agree(c, rc, COMM_MERGE_HOST, n_local, n_elems);
    if (rc || n_elems == 0) return rc;
    rc = allgather_fold_impl(c, c->comm_local.as<uint32_t>(), n_local, n_elems, c->comm_out.as<uint32_t>());
    if (!rc) rc = comm_finish(c, COMM_MERGE_HOST);
    if (rc) return rc;
    return comm_copy_out(c, host_out, n_elems * ebytes);
}

extern "C" int mastic_aggregate_merged(mastic_ctx* c, uint32_t agg_mask, const uint8_t* valid, size_t n_elems,
                                       uint8_t* agg_out) {
    DeviceScope ds_(c);
    if (!c) return MASTIC_EINVAL;
    const bool zeros = (agg_mask & MASTIC_MERGE_ZEROS) != 0;
    agg_mask &= ~MASTIC_MERGE_ZEROS;
    const size_t ebytes = (size_t)c->p.w32 * 4;
    const size_t n_local = (agg_mask & 1) + ((agg_mask >> 1) & 1);
    int rc = 0;
    if (agg_mask == 0 || agg_mask > 3) rc = fail(c, MASTIC_EINVAL, "invalid aggregator mask");
    if (!rc && n_elems && !agg_out) rc = fail(c, MASTIC_EINVAL, "null agg share buffer");
    if (!rc) rc = comm_check_counts(c, n_local, n_elems);
    for (int a = 0; a < 2 && !rc && n_elems && !zeros; a++) {
        if (!((agg_mask >> a) & 1)) continue;
        const Result& R = c->res[a];
        if (!R.ready)
            rc = fail(c, MASTIC_EINVAL, "no prep_init result for this aggregator");
        else if ((size_t)R.n_prefixes * (1 + c->p.output_len) != n_elems)
            rc = fail(c, MASTIC_EINVAL, "agg share length does not match the last prep_init");
    }
    if (!rc && n_elems &&
        (!comm_grow(c, c->comm_local, n_local * n_elems * ebytes) || !comm_grow(c, c->comm_out, n_elems * ebytes) ||
         !comm_stage_gather(c, n_local, n_elems)))
        rc = fail(c, MASTIC_ENOMEM, "out of device memory");
    size_t k = 0;
    for (int a = 0; a < 2 && !rc && n_elems; a++) {
        if (!((agg_mask >> a) & 1)) continue;
        uint32_t* dst = (uint32_t*)((uint8_t*)c->comm_local.p + k++ * n_elems * ebytes);
        if (!zeros)
            rc = aggregate_impl(c, a, valid, dst);
        else if (hipMemsetAsync(dst, 0, n_elems * ebytes, c->stream) != hipSuccess)  // no reports here: agg_init's zeros
            rc = fail(c, MASTIC_EHIP, "hipMemsetAsync failed");
    }
    rc = comm_agree(c, rc, COMM_AGGREGATE_MERGED, n_local, n_elems);
    if (rc || n_elems == 0) return rc;
    rc = allgather_fold_impl(c, c->comm_local.as<uint32_t>(), n_local, n_elems, c->comm_out.as<uint32_t>());
    if (!rc) rc = comm_finish(c, COMM_AGGREGATE_MERGED);
    if (rc) return rc;
    return comm_copy_out(c, agg_out, n_elems * ebytes);
}

// Eval-proof Merkle tree (proof-aggregation mode, kernels.hpp k_proof_tree_*)
// over the last prep_init result of agg_id.
extern "C" int mastic_proof_tree(mastic_ctx* c, int agg_id, const uint8_t* app_ctx, size_t ctx_len,
                                 uint8_t* nodes_out, size_t n_nodes) {
    DeviceScope ds_(c);
    if (!c || (agg_id != 0 && agg_id != 1)) return fail(c, MASTIC_EINVAL, "invalid aggregator ID");
    Result& R = c->res[agg_id];
    if (!R.ready) return fail(c, MASTIC_EINVAL, "no prep_init result for this aggregator");
    const size_t n = R.n;
    size_t total = 0;
    for (size_t m = n; m > 0; m = (m == 1) ? 0 : (m + 1) / 2) total += m;
    if (n_nodes != total) return fail(c, MASTIC_EINVAL, "proof tree has incorrect size");
    if (n == 0) return 0;
    if (n > (size_t)INT32_MAX / 2) return fail(c, MASTIC_EINVAL, "batch too large for a proof tree");
    int rc = build_prefixes(c, app_ctx, ctx_len, nullptr, 0);
    if (rc) return rc;
    DevBuf nodes;
    if (!nodes.ensure(total * 32)) return fail(c, MASTIC_ENOMEM, "out of device memory (proof tree)");
    uint32_t* d = nodes.as<uint32_t>();
    hipLaunchKernelGGL(k_proof_tree_leaves, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, c->stream,
                       R.eval_proof.as<uint32_t>(), (int)n, (int)R.stride, d);
    size_t off = 0;
    for (size_t m = n; m > 1; m = (m + 1) / 2) {
        const size_t mo = (m + 1) / 2;
        hipLaunchKernelGGL(k_proof_tree_level, dim3((unsigned)((mo + 255) / 256)), dim3(256), 0, c->stream,
                           (const PrefixState*)c->pfx.p, d + off * 8, (int)m, d + (off + m) * 8);
        off += m;
    }
    HIPCHK(c, hipGetLastError());
    HIPCHK(c, hipMemcpyAsync(nodes_out, d, total * 32, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    return 0;
}

extern "C" int mastic_synchronize(mastic_ctx* c) {
    DeviceScope ds_(c);
    if (!c) return MASTIC_EINVAL;
    HIPCHK(c, hipStreamSynchronize(c->stream));
    c->bury();
    return 0;
}

extern "C" int mastic_last_timing(mastic_ctx* c, double* eval_ms, int* eval_launches, double* absorb_ms,
                                  int* absorb_launches, double* total_ms) {
    return mastic_last_timing3(c, eval_ms, eval_launches, nullptr, nullptr, absorb_ms, absorb_launches, total_ms);
}

extern "C" int mastic_last_timing3(mastic_ctx* c, double* aes_ms, int* aes_launches, double* proof_ms,
                                   int* proof_launches, double* absorb_ms, int* absorb_launches, double* total_ms) {
    DeviceScope ds_(c);
    if (!c) return MASTIC_EINVAL;
    HIPCHK(c, hipStreamSynchronize(c->stream));
    if (c->tm[c->tcur].n_eval < 0) {
        // some timing marks sit on the sponge streams without the main stream
        // waiting for them (a single-chunk hit's empty sponge marks, recorded
        // on the sponge stream while its sponges run on the main stream):
        // wait for the marks themselves (an unwaited mark gave "device not
        // ready" in a 4-rank run sharing one GPU)
        if (!c->timing_nowait)
            for (int i = 0; i < -c->tm[c->tcur].n_eval; i++) HIPCHK(c, hipEventSynchronize(c->tm[c->tcur].ev[i]));
        // events: [t0, t1] then per level [aes0, aes1, proof0, proof1, absorb0, absorb1]
        const size_t evi = (size_t)(-c->tm[c->tcur].n_eval);
        double ta = 0, tp = 0, tb = 0;
        int n = 0;
        float ms = 0;
        for (size_t i = 2; i + 6 <= evi; i += 6) {
            HIPCHK(c, hipEventElapsedTime(&ms, c->tm[c->tcur].ev[i], c->tm[c->tcur].ev[i + 1]));
            ta += ms;
            HIPCHK(c, hipEventElapsedTime(&ms, c->tm[c->tcur].ev[i + 2], c->tm[c->tcur].ev[i + 3]));
            tp += ms;
            HIPCHK(c, hipEventElapsedTime(&ms, c->tm[c->tcur].ev[i + 4], c->tm[c->tcur].ev[i + 5]));
            tb += ms;
            n++;
        }
        HIPCHK(c, hipEventElapsedTime(&ms, c->tm[c->tcur].ev[0], c->tm[c->tcur].ev[1]));
        c->tm[c->tcur].t_total = ms;
        c->tm[c->tcur].t_eval = ta;
        c->tm[c->tcur].t_proof = tp;
        c->tm[c->tcur].t_absorb = tb;
        c->tm[c->tcur].n_eval = n;
        c->tm[c->tcur].n_absorb = n;
    }
    if (aes_ms) *aes_ms = c->tm[c->tcur].t_eval;
    if (aes_launches) *aes_launches = c->tm[c->tcur].n_eval;
    if (proof_ms) *proof_ms = c->tm[c->tcur].t_proof;
    if (proof_launches) *proof_launches = c->tm[c->tcur].n_absorb;
    if (absorb_ms) *absorb_ms = c->tm[c->tcur].t_absorb;
    if (absorb_launches) *absorb_launches = c->tm[c->tcur].n_absorb;
    if (total_ms) *total_ms = c->tm[c->tcur].t_total;
    return 0;
}

extern "C" int mastic_tree_stats(mastic_ctx* c, const uint8_t* enc, size_t len, uint64_t* nodes, uint64_t* interior,
                                 uint64_t* max_level_nodes) {
    DeviceScope ds_(c);
    Tree* t = nullptr;
    int rc = build_tree(c, enc, len, &t);
    if (rc) return rc;
    if (nodes) *nodes = t->nodes;
    if (interior) *interior = t->interior;
    if (max_level_nodes) *max_level_nodes = (uint64_t)t->max_level_nodes;
    return 0;
}

extern "C" int mastic_work_bytes(mastic_ctx* c, const uint8_t* enc, size_t len, uint64_t* per_report) {
    DeviceScope ds_(c);
    Tree* t = nullptr;
    int rc = build_tree(c, enc, len, &t);
    if (rc) return rc;
    if (per_report) *per_report = (uint64_t)work_layout(c->p, t).words * 4;
    return 0;
}

extern "C" int mastic_prep_init_batch(mastic_ctx* c, const uint8_t* verify_key, size_t vk_len, const uint8_t* app_ctx,
                                      size_t ctx_len, int agg_id, const uint8_t* enc_agg_param, size_t agg_param_len,
                                      size_t n, const uint8_t* nonces, const uint8_t* public_shares,
                                      const uint8_t* input_shares, uint8_t* prep_shares_out, uint8_t* jr_seeds_out,
                                      uint8_t* out_shares_out, int32_t* status_out) {
    DeviceScope ds_(c);
    if (!c) return MASTIC_EINVAL;
    if (agg_id != 0 && agg_id != 1) return fail(c, MASTIC_EINVAL, "invalid aggregator ID");
    mastic_reports* rep = nullptr;
    int rc = mastic_reports_create(c, n, &rep);
    if (rc) return rc;
    rc = mastic_reports_upload(rep, nonces, public_shares, agg_id == 0 ? input_shares : nullptr,
                               agg_id == 1 ? input_shares : nullptr);
    if (!rc) rc = mastic_prep_init(c, rep, verify_key, vk_len, app_ctx, ctx_len, agg_id, enc_agg_param, agg_param_len);
    if (!rc) rc = mastic_prep_result(c, agg_id, prep_shares_out, jr_seeds_out, out_shares_out, status_out);
    mastic_reports_destroy(rep);
    return rc;
}

// ---------------------------------------------------------------- decide
extern "C" int mastic_decide_batch(mastic_ctx* c, const uint8_t* app_ctx, size_t ctx_len, const uint8_t* enc,
                                   size_t len, size_t n, const uint8_t* ps0, const uint8_t* ps1, uint8_t* msgs_out,
                                   uint8_t* valid_out) {
    DeviceScope ds_(c);
    if (!c) return MASTIC_EINVAL;
    Tree* t = nullptr;
    int rc = build_tree(c, enc, len, &t);
    if (rc) return rc;
    if (n == 0) return 0;
    if ((rc = build_prefixes(c, app_ctx, ctx_len, nullptr, 0))) return rc;
    const McParams& p = c->p;
    const size_t psz = mc_prep_share_size(p, t->weight_check);
    const size_t stride = round_up(n, 64);
    DevBuf a, b, ver, msg, st;
    if (!a.ensure(psz * n) || !b.ensure(psz * n) || !ver.ensure(stride * 4 * (size_t)p.verifier_len * p.w32) ||
        !msg.ensure(32 * n) || !st.ensure(n))
        return fail(c, MASTIC_ENOMEM, "out of device memory (decide)");
    HIPCHK(c, hipMemcpyAsync(a.p, ps0, psz * n, hipMemcpyHostToDevice, c->stream));
    HIPCHK(c, hipMemcpyAsync(b.p, ps1, psz * n, hipMemcpyHostToDevice, c->stream));
    HIPCHK(c, hipMemsetAsync(msg.p, 0, 32 * n, c->stream));
    if (p.field == 64)
        hipLaunchKernelGGL(k_decide<F64>, dim3((n + 255) / 256), dim3(256), 0, c->stream, p, (int)n, (int)stride,
                           (int)t->weight_check, a.as<uint8_t>(), b.as<uint8_t>(), (int)psz, ver.as<uint32_t>(),
                           (const PrefixState*)c->pfx.p, msg.as<uint8_t>(), st.as<uint8_t>());
    else
        hipLaunchKernelGGL(k_decide<F128>, dim3((n + 255) / 256), dim3(256), 0, c->stream, p, (int)n, (int)stride,
                           (int)t->weight_check, a.as<uint8_t>(), b.as<uint8_t>(), (int)psz, ver.as<uint32_t>(),
                           (const PrefixState*)c->pfx.p, msg.as<uint8_t>(), st.as<uint8_t>());
    HIPCHK(c, hipGetLastError());
    if (msgs_out && t->weight_check && p.joint_rand_len > 0)
        HIPCHK(c, hipMemcpyAsync(msgs_out, msg.p, 32 * n, hipMemcpyDeviceToHost, c->stream));
    if (valid_out) HIPCHK(c, hipMemcpyAsync(valid_out, st.p, n, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    return 0;
}

// ---------------------------------------------------------------- reports
extern "C" int mastic_reports_create(mastic_ctx* c, size_t n, mastic_reports** out) {
    DeviceScope ds_(c);
    if (!c || !out) return MASTIC_EINVAL;
    mastic_reports* r = new mastic_reports();
    r->ctx = c;
    r->n = n;
    const McParams& p = c->p;
    if (!r->nonces.ensure(16 * n) || !r->pub.ensure((size_t)mc_public_share_size(p) * n)) {
        delete r;
        return fail(c, MASTIC_ENOMEM, "out of device memory (reports)");
    }
    *out = r;
    return 0;
}

extern "C" int mastic_reports_view(mastic_reports* rep, size_t first, size_t count, mastic_reports** out) {
    DeviceScope ds_(rep ? rep->ctx : nullptr);
    if (!rep || !out) return MASTIC_EINVAL;
    mastic_ctx* c = rep->ctx;
    if (first > rep->n || count > rep->n - first) return fail(c, MASTIC_EINVAL, "view out of range");
    const McParams& p = c->p;
    mastic_reports* r = new mastic_reports();
    r->ctx = c;
    r->n = count;
    r->gen = rep->gen;  // one contents generation for the batch and all its views
    const size_t ps = mc_public_share_size(p), i0 = mc_input_share_size(p, 0), i1 = mc_input_share_size(p, 1);
    r->nonces.view(rep->nonces, 16 * first, 16 * count);
    r->pub.view(rep->pub, ps * first, ps * count);
    r->in0.view(rep->in0, i0 * first, i0 * count);
    r->in1.view(rep->in1, i1 * first, i1 * count);
    *out = r;
    return 0;
}

extern "C" void mastic_reports_destroy(mastic_reports* r) {
    DeviceScope ds_(r ? r->ctx : nullptr);
    delete r;
}
extern "C" size_t mastic_reports_count(const mastic_reports* r) { return r ? r->n : 0; }

extern "C" int mastic_reports_upload(mastic_reports* r, const uint8_t* nonces, const uint8_t* pub,
                                     const uint8_t* in0, const uint8_t* in1) {
    DeviceScope ds_(r ? r->ctx : nullptr);
    if (!r) return MASTIC_EINVAL;
    mastic_ctx* c = r->ctx;
    const McParams& p = c->p;
    const size_t n = r->n;
    r->touch();
    if (nonces) HIPCHK(c, hipMemcpy(r->nonces.p, nonces, 16 * n, hipMemcpyHostToDevice));
    if (pub) HIPCHK(c, hipMemcpy(r->pub.p, pub, (size_t)mc_public_share_size(p) * n, hipMemcpyHostToDevice));
    if (in0) {
        if (!r->in0.ensure((size_t)mc_input_share_size(p, 0) * n)) return fail(c, MASTIC_ENOMEM, "out of device memory");
        HIPCHK(c, hipMemcpy(r->in0.p, in0, (size_t)mc_input_share_size(p, 0) * n, hipMemcpyHostToDevice));
    }
    if (in1) {
        if (!r->in1.ensure((size_t)mc_input_share_size(p, 1) * n)) return fail(c, MASTIC_ENOMEM, "out of device memory");
        HIPCHK(c, hipMemcpy(r->in1.p, in1, (size_t)mc_input_share_size(p, 1) * n, hipMemcpyHostToDevice));
    }
    return 0;
}

extern "C" int mastic_reports_download(mastic_reports* r, uint8_t* nonces, uint8_t* pub, uint8_t* in0, uint8_t* in1) {
    DeviceScope ds_(r ? r->ctx : nullptr);
    if (!r) return MASTIC_EINVAL;
    mastic_ctx* c = r->ctx;
    const McParams& p = c->p;
    const size_t n = r->n;
    HIPCHK(c, hipStreamSynchronize(c->stream));
    if (nonces) HIPCHK(c, hipMemcpy(nonces, r->nonces.p, 16 * n, hipMemcpyDeviceToHost));
    if (pub) HIPCHK(c, hipMemcpy(pub, r->pub.p, (size_t)mc_public_share_size(p) * n, hipMemcpyDeviceToHost));
    if (in0) {
        if (!r->in0.p) return fail(c, MASTIC_EINVAL, "no leader input shares");
        HIPCHK(c, hipMemcpy(in0, r->in0.p, (size_t)mc_input_share_size(p, 0) * n, hipMemcpyDeviceToHost));
    }
    if (in1) {
        if (!r->in1.p) return fail(c, MASTIC_EINVAL, "no helper input shares");
        HIPCHK(c, hipMemcpy(in1, r->in1.p, (size_t)mc_input_share_size(p, 1) * n, hipMemcpyDeviceToHost));
    }
    return 0;
}

template <class F>
static int shard_impl(mastic_ctx* c, mastic_reports* rep, const uint8_t* alphas, const uint8_t* betas,
                      const uint8_t* nonces, const uint8_t* rands) {
    typedef typename F::E E;
    const McParams& p = c->p;
    const size_t n = rep->n;
    const size_t ab = (p.bits + 7) / 8, bsz = (size_t)p.meas_len * p.enc, rs = mc_rand_size(p);
    if (!rep->in0.ensure((size_t)mc_input_share_size(p, 0) * n) || !rep->in1.ensure((size_t)mc_input_share_size(p, 1) * n))
        return fail(c, MASTIC_ENOMEM, "out of device memory (input shares)");
    DevBuf da, db, dr, tab;
    if (!da.ensure(ab * n) || !db.ensure(bsz * n) || !dr.ensure(rs * n) || !tab.ensure(sizeof(E) * p.P))
        return fail(c, MASTIC_ENOMEM, "out of device memory (shard inputs)");
    HIPCHK(c, hipMemcpy(da.p, alphas, ab * n, hipMemcpyHostToDevice));
    HIPCHK(c, hipMemcpy(db.p, betas, bsz * n, hipMemcpyHostToDevice));
    HIPCHK(c, hipMemcpy(dr.p, rands, rs * n, hipMemcpyHostToDevice));
    HIPCHK(c, hipMemcpy(rep->nonces.p, nonces, 16 * n, hipMemcpyHostToDevice));
    FlpConsts<F> fc = flp_consts<F>(p);
    std::vector<E> pows(p.P);
    E ainv = finv<F>(fc.alpha), acc = F::from_u64(1);
    for (int i = 0; i < p.P; i++) {
        pows[i] = acc;
        acc = F::mul(acc, ainv);
    }
    HIPCHK(c, hipMemcpy(tab.p, pows.data(), sizeof(E) * p.P, hipMemcpyHostToDevice));
    // scratch planes per report
    const size_t wl = (size_t)p.value_len * p.w32;
    const size_t words = wl + 88 + 2 * wl + (size_t)std::max(1, p.joint_rand_len) * p.w32 + (size_t)p.arity * p.w32 +
                         2 * (size_t)p.arity * p.P * p.w32 + 2 * (size_t)p.proof_len * p.w32 + 32;
    const uint64_t budget = default_budget(c);
    size_t chunk = std::min<size_t>(round_up(n, 64), std::max<size_t>(64, (budget / (words * 4)) / 64 * 64));
    // the scratch is the ctx's work arena (kept across calls, stream-ordered
    // after earlier prep_inits): sharding a large batch leaves the arena that
    // its prep_inits then reuse instead of freeing it and allocating again
    // (large hipMallocs / hipFrees cost ~1 s per 50-100 GB on MI355X)
    DevBuf& scratch = c->work;
    c->rk.valid = false;  // the scratch overwrites the arena's key-schedule planes
    if (!scratch.ensure(words * 4 * chunk)) return fail(c, MASTIC_ENOMEM, "out of device memory (shard scratch)");
    for (size_t b = 0; b < n; b += chunk) {
        const int nn = (int)std::min(chunk, n - b);
        const int S = (int)round_up(nn, 64);
        ShardArgs a;
        a.n = nn;
        a.stride = S;
        a.alphas = da.as<uint8_t>() + ab * b;
        a.betas = db.as<uint8_t>() + bsz * b;
        a.nonces = rep->nonces.as<uint8_t>() + 16 * b;
        a.rands = dr.as<uint8_t>() + rs * b;
        a.pub = rep->pub.as<uint8_t>() + (size_t)mc_public_share_size(p) * b;
        a.in0 = rep->in0.as<uint8_t>() + (size_t)mc_input_share_size(p, 0) * b;
        a.in1 = rep->in1.as<uint8_t>() + (size_t)mc_input_share_size(p, 1) * b;
        uint32_t* w = scratch.as<uint32_t>();
        size_t o = 0;
        auto take = [&](size_t k) {
            uint32_t* r = w + o * S;
            o += k;
            return r;
        };
        a.beta = take(wl);
        a.rke = take(44);
        a.rkc = take(44);
        a.bs = take(2 * wl);
        a.jr = take((size_t)std::max(1, p.joint_rand_len) * p.w32);
        a.prand = take((size_t)p.arity * p.w32);
        a.vals = take((size_t)p.arity * p.P * p.w32);
        a.coef = take((size_t)p.arity * p.P * p.w32);
        a.proof = take((size_t)p.proof_len * p.w32);
        a.hps = take((size_t)p.proof_len * p.w32);
        a.misc = take(32);
        hipLaunchKernelGGL(k_shard<F>, dim3((nn + 255) / 256), dim3(256), 0, c->stream, p, a,
                           (const PrefixState*)c->pfx.p, fc, tab.as<E>());
        HIPCHK(c, hipGetLastError());
    }
    HIPCHK(c, hipStreamSynchronize(c->stream));
    return 0;
}

extern "C" int mastic_reports_shard(mastic_reports* rep, const uint8_t* app_ctx, size_t ctx_len,
                                    const uint8_t* alphas, const uint8_t* betas, const uint8_t* nonces,
                                    const uint8_t* rands) {
    DeviceScope ds_(rep ? rep->ctx : nullptr);
    if (!rep) return MASTIC_EINVAL;
    mastic_ctx* c = rep->ctx;
    rep->touch();
    if (rep->n == 0) {
        // an empty batch holds both aggregators' (zero) input shares, so that
        // prep_init accepts it and its views (e.g. a rank of a split job that
        // gets no reports)
        if (!rep->in0.ensure(0) || !rep->in1.ensure(0)) return fail(c, MASTIC_ENOMEM, "out of device memory");
        return 0;
    }
    if (!alphas || !nonces || !rands || (!betas && c->p.meas_len > 0)) return fail(c, MASTIC_EINVAL, "null input");
    int rc = build_prefixes(c, app_ctx, ctx_len, nullptr, 0);
    if (rc) return rc;
    return c->p.field == 64 ? shard_impl<F64>(c, rep, alphas, betas, nonces, rands)
                            : shard_impl<F128>(c, rep, alphas, betas, nonces, rands);
}

extern "C" int mastic_shard_batch(mastic_ctx* c, const uint8_t* app_ctx, size_t ctx_len, size_t n,
                                  const uint8_t* alphas, const uint8_t* betas, const uint8_t* nonces,
                                  const uint8_t* rands, uint8_t* pub_out, uint8_t* in0_out, uint8_t* in1_out) {
    DeviceScope ds_(c);
    if (!c) return MASTIC_EINVAL;
    mastic_reports* rep = nullptr;
    int rc = mastic_reports_create(c, n, &rep);
    if (rc) return rc;
    rc = mastic_reports_shard(rep, app_ctx, ctx_len, alphas, betas, nonces, rands);
    if (!rc) rc = mastic_reports_download(rep, nullptr, pub_out, in0_out, in1_out);
    mastic_reports_destroy(rep);
    return rc;
}

// ---------------------------------------------------------------- ctx
extern "C" int mastic_ctx_create(const mastic_params* up, mastic_ctx** out) {
    if (!up || !out) return MASTIC_EINVAL;
    *out = nullptr;
    McParams p;
    if (mc_derive((int)up->circuit, (int)up->bits, (int)up->length, (int)up->sum_vec_bits, up->max_measurement,
                  (int)up->chunk_length, &p))
        return MASTIC_EINVAL;
    if (p.bits > TREE_MAX_BITS) return MASTIC_EINVAL;  // node paths are at most 256 bits (host_tree.hpp)
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) return MASTIC_ENODEV;
    if (up->device < 0 || up->device >= ndev) return MASTIC_ENODEV;
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, up->device) != hipSuccess) return MASTIC_ENODEV;
    if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0) return MASTIC_ENODEV;
    if (hipSetDevice(up->device) != hipSuccess) return MASTIC_ENODEV;
    mastic_ctx* c = new mastic_ctx();
    c->user = *up;
    c->p = p;
    c->device = up->device;
    c->n_cus = prop.multiProcessorCount > 0 ? prop.multiProcessorCount : 256;
    {
        int khz = 0;
        if (hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, up->device) == hipSuccess && khz > 0)
            c->wall_khz = khz;
    }
#ifdef MASTIC_EXPERIMENT_KNOBS
    // A/B and timing experiments only (tools/ab_*.sh build the library with
    // -DMASTIC_EXPERIMENT_KNOBS; the shipped library reads none of these).
    // MASTIC_DBG_SKIP and MASTIC_ABSORB_DBG skip or gut kernels: results wrong.
    {
        const char* e = getenv("MASTIC_ABSORB_SINGLE");
        if (e) c->absorb_mode = e[0] == '1' ? 1 : (e[0] == '2' ? 2 : 0);
        const char* esm = getenv("MASTIC_ABSORB_SINGLE_MIN");
        if (esm) c->absorb_single_min = (size_t)std::max(0, atoi(esm));
        const char* l = getenv("MASTIC_ABSORB_LDS_KB");
        c->absorb_lds = l ? std::max(0, std::min(160, atoi(l))) * 1024 : 0;
        const char* pw = getenv("MASTIC_PROOF_WAVES");
        if (pw) c->proof_waves = std::max(1, std::min(15, atoi(pw)));
        const char* spd = getenv("MASTIC_STRIDE_PAD");
        if (spd) c->stride_pad = std::max(0, std::min(1 << 20, atoi(spd))) / 64 * 64;
        const char* wa = getenv("MASTIC_WORK_ARENA_GB");
        if (wa) c->work_arena = c->work_arena_fc = (size_t)std::max(0, atoi(wa)) << 30;
        const char* bt = getenv("MASTIC_BINDER_TILED");
        if (bt) c->binder_tiled = bt[0] != '0';
        const char* at = getenv("MASTIC_ABSORB_THREADS");
        if (at) c->absorb_threads = std::max(64, std::min(256, atoi(at))) / 64 * 64;
        const char* ap = getenv("MASTIC_ABSORB_PRIO");
        if (ap) c->absorb_prio = std::max(0, std::min(3, atoi(ap)));
        const char* adb = getenv("MASTIC_ABSORB_DBG");
        if (adb) c->absorb_dbg = atoi(adb);
        const char* dsk = getenv("MASTIC_DBG_SKIP");
        if (dsk) c->dbg_skip = atoi(dsk);
        const char* xp = getenv("MASTIC_AES_PRIO");
        if (xp) c->aes_prio = std::max(0, std::min(2, atoi(xp)));
        const char* pp = getenv("MASTIC_PROOF_PRIO");
        if (pp) c->proof_prio = std::max(0, std::min(2, atoi(pp)));
        const char* pw2 = getenv("MASTIC_PAR_WAVES");
        if (pw2) c->par_waves = std::max(1, std::min(EVAL_WAVES, atoi(pw2)));
        const char* cp = getenv("MASTIC_CHUNK_PIPELINE");
        if (cp) c->chunk_pipeline = cp[0] != '0';
        const char* hpw = getenv("MASTIC_HIT_PROOF_WAVES");
        if (hpw) c->hit_proof_waves = std::max(0, std::min(15, atoi(hpw)));
        const char* fp = getenv("MASTIC_FUSE_PROOFS");
        if (fp) c->fuse_proofs = std::max(0, std::min(3, atoi(fp)));
        const char* fa = getenv("MASTIC_FC_ALL");
        if (fa) c->fc_all = fa[0] == '1';
        const char* cr = getenv("MASTIC_CHUNK_REPORTS");
        if (cr) c->chunk_max = (size_t)std::max(0, atoi(cr));
        const char* spl = getenv("MASTIC_SPLIT_SPONGES");
        if (spl) c->split_sponges = spl[0] == '1' ? 1 : 0;
        const char* flm = getenv("MASTIC_FUSE_LAST_MISS");
        if (flm) c->fuse_last_miss = flm[0] == '1';
        const char* flf = getenv("MASTIC_FUSE_LAST_MISS_FC");
        if (flf) c->fuse_last_miss_fc = flf[0] != '0';
        const char* ham = getenv("MASTIC_HIT_ABSORB_MAIN");
        if (ham) c->hit_absorb_main = ham[0] != '0';
        const char* ssp = getenv("MASTIC_SMALL_SPLIT");
        if (ssp) c->small_split = ssp[0] != '0';
        const char* tnw = getenv("MASTIC_DBG_TIMING_NOWAIT");  // the round-5 last_timing bug, for its test's A/B
        if (tnw) c->timing_nowait = tnw[0] == '1';
        const char* ssr = getenv("MASTIC_SERIAL_SPONGES");
        if (ssr) c->serial_sponges = ssr[0] == '1';
    }
#endif
    // the level kernel's LDS (table + key schedules) is dynamic, above the
    // 64 KiB default
    if (hipFuncSetAttribute((const void*)k_eval_aes<F64, false, false>, hipFuncAttributeMaxDynamicSharedMemorySize,
                            EVAL_LDS_BYTES) != hipSuccess ||
        hipFuncSetAttribute((const void*)k_eval_aes<F128, false, false>, hipFuncAttributeMaxDynamicSharedMemorySize,
                            EVAL_LDS_BYTES) != hipSuccess ||
        hipFuncSetAttribute((const void*)k_eval_aes<F64, true, false>, hipFuncAttributeMaxDynamicSharedMemorySize,
                            EVAL_LDS_BYTES) != hipSuccess ||
        hipFuncSetAttribute((const void*)k_eval_aes<F128, true, false>, hipFuncAttributeMaxDynamicSharedMemorySize,
                            EVAL_LDS_BYTES) != hipSuccess ||
        hipFuncSetAttribute((const void*)k_eval_aes<F64, true, true>, hipFuncAttributeMaxDynamicSharedMemorySize,
                            EVAL_LDS_BYTES) != hipSuccess ||
        hipFuncSetAttribute((const void*)k_eval_aes<F128, true, true>, hipFuncAttributeMaxDynamicSharedMemorySize,
                            EVAL_LDS_BYTES) != hipSuccess ||
        hipFuncSetAttribute((const void*)k_eval_aes<F64, true, false, true>,
                            hipFuncAttributeMaxDynamicSharedMemorySize, EVAL_LDS_BYTES) != hipSuccess ||
        hipFuncSetAttribute((const void*)k_eval_aes<F64, false, false, true>,
                            hipFuncAttributeMaxDynamicSharedMemorySize, EVAL_LDS_BYTES) != hipSuccess ||
        hipFuncSetAttribute((const void*)k_eval_aes<F128, true, false, true>,
                            hipFuncAttributeMaxDynamicSharedMemorySize, EVAL_LDS_BYTES) != hipSuccess ||
        hipFuncSetAttribute((const void*)k_eval_aes<F128, false, false, true>,
                            hipFuncAttributeMaxDynamicSharedMemorySize, EVAL_LDS_BYTES) != hipSuccess ||
        hipFuncSetAttribute((const void*)k_absorb_pair, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024) !=
            hipSuccess ||
        hipFuncSetAttribute((const void*)k_absorb, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024) !=
            hipSuccess) {
        delete c;
        return MASTIC_EHIP;
    }
    // the binder sponges are the latency-critical chain: their stream gets the
    // highest priority so their workgroups are dispatched first
    int prio_lo = 0, prio_hi = 0;
    (void)hipDeviceGetStreamPriorityRange(&prio_lo, &prio_hi);
    if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess ||
        hipStreamCreateWithPriority(&c->stream2, hipStreamNonBlocking, prio_hi) != hipSuccess ||
        hipStreamCreateWithPriority(&c->stream3, hipStreamNonBlocking, prio_hi) != hipSuccess ||
        hipStreamCreateWithFlags(&c->stream4, hipStreamNonBlocking) != hipSuccess) {
        delete c;
        return MASTIC_EHIP;
    }
    *out = c;
    return 0;
}

extern "C" void mastic_ctx_destroy(mastic_ctx* c) {
    DeviceScope ds_(c);
    if (!c) return;
    (void)hipStreamSynchronize(c->stream);
    (void)hipStreamSynchronize(c->stream2);
    (void)hipStreamSynchronize(c->stream3);
    (void)hipStreamSynchronize(c->stream4);
    delete c;
}

extern "C" const char* mastic_last_error(const mastic_ctx* c) { return c ? c->err.c_str() : "null ctx"; }

extern "C" int mastic_set_frontier_cache(mastic_ctx* c, int on, int* last_hit) {
    DeviceScope ds_(c);
    if (!c) return MASTIC_EINVAL;
    if (on >= 0) {
        c->frontier_cache = on != 0;
        if (!on) {
            // queued kernels may still read the cache slots: retire them (freed
            // at the next idle point of the ctx's streams), no synchronisation
            for (auto& x : c->lc) {
                for (DevBuf* b : {&x.sp, &x.rootsum, &x.nd}) {
                    if (b->p && b->own) c->graveyard.push_back(b->p);
                    b->p = nullptr;
                    b->bytes = 0;
                }
                x.release();
            }
            if (c->fc_spare.p && c->fc_spare.own) c->graveyard.push_back(c->fc_spare.p);
            c->fc_spare.p = nullptr;
            c->fc_spare.bytes = 0;
            c->spare_cap = 0;
            c->spare_S = 0;
        }
    }
    if (last_hit) *last_hit = c->last_hit ? 1 : 0;
    return 0;
}

extern "C" int mastic_set_test_hooks(mastic_ctx* c, int force_slow_blk, int fail_allocs) {
    if (!c) return MASTIC_EINVAL;
    const int pending = c->fail_allocs;
    c->force_slow_blk = force_slow_blk < 0 ? -1 : force_slow_blk;
    c->fail_allocs = std::max(0, fail_allocs);
    return pending;
}

extern "C" int mastic_set_serial_sponges(mastic_ctx* c, int on) {
    if (!c) return MASTIC_EINVAL;
    const int prev = c->serial_sponges ? 1 : 0;
    if (on >= 0) c->serial_sponges = on != 0;
    return prev;
}

extern "C" int mastic_set_test_sponge_delay(mastic_ctx* c, int delay_us) {
    if (!c || delay_us < 0 || delay_us > 10000000) return MASTIC_EINVAL;
    c->sponge_delay_us = delay_us;
    return 0;
}

extern "C" int mastic_abi_version(void) { return MASTIC_ABI_VERSION; }

extern "C" int mastic_set_memory_budget(mastic_ctx* c, uint64_t bytes) {
    if (!c) return MASTIC_EINVAL;
    c->budget = bytes;
    return 0;
}

extern "C" int mastic_get_sizes(const mastic_ctx* c, mastic_sizes* s) {
    if (!c || !s) return MASTIC_EINVAL;
    const McParams& p = c->p;
    s->field_bytes = p.enc;
    s->value_len = p.value_len;
    s->meas_len = p.meas_len;
    s->output_len = p.output_len;
    s->proof_len = p.proof_len;
    s->verifier_len = p.verifier_len;
    s->joint_rand_len = p.joint_rand_len;
    s->query_rand_len = p.query_rand_len;
    s->prove_rand_len = p.prove_rand_len;
    s->rand_size = mc_rand_size(p);
    s->public_share_size = mc_public_share_size(p);
    s->input_share_size[0] = mc_input_share_size(p, 0);
    s->input_share_size[1] = mc_input_share_size(p, 1);
    s->prep_share_size[0] = mc_prep_share_size(p, false);
    s->prep_share_size[1] = mc_prep_share_size(p, true);
    s->algorithm_id = p.alg_id;
    return 0;
}
