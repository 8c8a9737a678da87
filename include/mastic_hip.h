/*
 * mastic_hip.h — C ABI of the MI355X (gfx950) batched Mastic aggregator.
 *
 * Drop-in boundary for the reference's per-report Mastic API
 * (poc/mastic.py, class Mastic :52-559, instantiations :567-614).  Every
 * entry point is batch-first: it processes n reports that share one
 * aggregation parameter, with caller-owned buffers holding the reference's
 * wire encodings (test_vec/mastic format).  Plain pointers and sizes only.
 *
 *   reference (poc/)                         replaced by
 *   ------------------------------------------------------------------
 *   Mastic.__init__ / MasticCount.. :81-89,   mastic_ctx_create
 *       :567-614
 *   Mastic.shard :91-185                      mastic_shard_batch,
 *   (Vidpf.gen vidpf.py:103-211)              mastic_reports_shard
 *   Mastic.prep_init :205-318                 mastic_prep_init_batch,
 *   (Vidpf.eval_with_siblings :213-261,       mastic_prep_init +
 *    FlpBBCGGI19.query)                       mastic_prep_result
 *   Mastic.prep_shares_to_prep :320-362       mastic_decide_batch
 *   (FlpBBCGGI19.decide)
 *   Mastic.agg_init/agg_update/merge          mastic_aggregate
 *       :379-397
 *   Mastic.encode_agg_param :413-435          (consumed as input, decoded here)
 *
 * Errors: 0 on success, a negative MASTIC_E* code otherwise (the reference's
 * ValueError cases map to MASTIC_EINVAL; mastic_last_error() gives the text).
 * Per-report verification outcomes are reported in status arrays instead of
 * raising.  Calls block until their results are in the caller's buffers
 * (mastic_prep_init is the exception: it only enqueues).  A ctx is
 * thread-compatible, not thread-safe.  The library never frees caller memory.
 *
 * The product path has no CPU fallback: without a usable gfx950 device
 * mastic_ctx_create fails with MASTIC_ENODEV.
 */
#ifndef MASTIC_HIP_H
#define MASTIC_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ABI version of this header; mastic_abi_version() returns the library's.
 * 4: mastic_aggregate_device_on_stream, mastic_set_test_hooks.
 * 5: mastic_aggregate_device takes the caller's stream again (its round-3,
 *    pre-versioning signature; ABI 4 had briefly dropped it), the
 *    library-owned RCCL communicator (mastic_comm_*, mastic_allgather_fold,
 *    mastic_aggregate_merged).
 * 6: collective-safe merges (an agreement round before any share moves,
 *    bounded waits, MASTIC_ETIMEDOUT), mastic_comm_init_timeout, RCCL bound at
 *    run time (no load-time librccl dependency); the old entry point
 *    mastic_aggregate_device is removed -- its argument count changed
 *    between ABI 3, 4 and 5 -- and the stream form is
 *    mastic_aggregate_device_on_stream only, so a binary built against an
 *    older header fails to link instead of passing a garbage stream;
 *    mastic_set_serial_sponges (measurement schedule), mastic_set_test_sponge_delay
 *    (test hook). */
#define MASTIC_ABI_VERSION 6

#define MASTIC_OK 0
#define MASTIC_EINVAL (-22)
#define MASTIC_ENOMEM (-12)
#define MASTIC_ENODEV (-19)
#define MASTIC_EHIP (-5)
#define MASTIC_ETIMEDOUT (-110) /* a peer rank did not join a collective step in time */

/* circuit ids = low byte of the reference's algorithm IDs (mastic.py:568-611) */
#define MASTIC_COUNT 1            /* MasticCount(bits)                         */
#define MASTIC_SUM 2              /* MasticSum(bits, max_measurement)          */
#define MASTIC_SUMVEC 3           /* MasticSumVec(bits, length, bits, chunk)   */
#define MASTIC_HISTOGRAM 4        /* MasticHistogram(bits, length, chunk)      */
#define MASTIC_MULTIHOT 5         /* MasticMultihotCountVec(bits, len, max_w, chunk) */

typedef struct mastic_params {
    uint32_t circuit;
    uint32_t bits;            /* VIDPF BITS */
    uint32_t length;          /* SumVec / Histogram / MultihotCountVec length */
    uint32_t sum_vec_bits;    /* SumVec bits */
    uint64_t max_measurement; /* Sum max_measurement / MultihotCountVec max_weight */
    uint32_t chunk_length;    /* SumVec / Histogram / MultihotCountVec chunk_length */
    int32_t device;           /* HIP device ordinal */
} mastic_params;

typedef struct mastic_sizes {
    uint32_t field_bytes;       /* ENCODED_SIZE: 8 (Field64) or 16 (Field128) */
    uint32_t value_len;         /* VIDPF VALUE_LEN = 1 + MEAS_LEN */
    uint32_t meas_len;
    uint32_t output_len;
    uint32_t proof_len;
    uint32_t verifier_len;
    uint32_t joint_rand_len;
    uint32_t query_rand_len;
    uint32_t prove_rand_len;
    uint32_t rand_size;         /* Mastic.RAND_SIZE */
    uint32_t public_share_size;
    uint32_t input_share_size[2];
    uint32_t prep_share_size[2]; /* [0] without, [1] with the weight check */
    uint32_t algorithm_id;
} mastic_sizes;

typedef struct mastic_ctx mastic_ctx;
typedef struct mastic_reports mastic_reports;

int mastic_ctx_create(const mastic_params* params, mastic_ctx** out);
void mastic_ctx_destroy(mastic_ctx* ctx);
const char* mastic_last_error(const mastic_ctx* ctx);
int mastic_get_sizes(const mastic_ctx* ctx, mastic_sizes* out);
/* Device-memory budget (bytes) for one prep_init batch's work buffers; 0 = default. */
int mastic_set_memory_budget(mastic_ctx* ctx, uint64_t bytes);

/* ---- reports resident in HBM (wire encodings, report-major) ---------- */
int mastic_reports_create(mastic_ctx* ctx, size_t n, mastic_reports** out);
void mastic_reports_destroy(mastic_reports* rep);
size_t mastic_reports_count(const mastic_reports* rep);
/* nonces n*16, public_shares n*public_share_size, input_shares{0,1}
 * n*input_share_size[agg]; either input-share pointer may be NULL. */
int mastic_reports_upload(mastic_reports* rep, const uint8_t* nonces, const uint8_t* public_shares,
                          const uint8_t* input_shares0, const uint8_t* input_shares1);
int mastic_reports_download(mastic_reports* rep, uint8_t* nonces, uint8_t* public_shares,
                            uint8_t* input_shares0, uint8_t* input_shares1);
/* A batch of `count` reports starting at report `first` of `rep`, sharing its
 * HBM (no copy).  It must be destroyed before `rep`; writing to either
 * (upload / shard) changes both. */
int mastic_reports_view(mastic_reports* rep, size_t first, size_t count, mastic_reports** out);
/* Client shard on the GPU (Mastic.shard).  alphas n*ceil(bits/8) MSB-first,
 * betas n*meas_len*field_bytes = the FLP-encoded measurement (Valid.encode),
 * nonces n*16, rands n*rand_size. */
int mastic_reports_shard(mastic_reports* rep, const uint8_t* app_ctx, size_t ctx_len, const uint8_t* alphas,
                         const uint8_t* betas, const uint8_t* nonces, const uint8_t* rands);

/* ---- aggregator preparation ----------------------------------------- */
/* Enqueue prep_init for every report of `rep` as aggregator agg_id.
 * verify_key is verify_key_len (0..255) bytes: it is XofTurboShake128's seed
 * (length-prefixed, mastic.py:302-306,499-510), so the reference driver's
 * 16-byte key (examples.py:38,176) and VERIFY_KEY_SIZE = 32 both work.
 * enc_agg_param is Mastic.encode_agg_param's output.  Results stay in HBM
 * (one result slot per agg_id) until read or aggregated. */
int mastic_prep_init(mastic_ctx* ctx, mastic_reports* rep, const uint8_t* verify_key, size_t verify_key_len,
                     const uint8_t* app_ctx, size_t ctx_len, int agg_id, const uint8_t* enc_agg_param,
                     size_t agg_param_len);
/* Copy results of the last mastic_prep_init for agg_id (blocks).  Any output
 * may be NULL.  prep_shares n*prep_share_size[weight_check] (wire encoding,
 * mastic.py:543-552); jr_seeds n*32 (zero when not applicable);
 * out_shares n*len(prefixes)*(1+output_len)*field_bytes (truncated output
 * shares = prep_state[0], encode_vec); status n (0 = ok, <0 = query abort). */
int mastic_prep_result(mastic_ctx* ctx, int agg_id, uint8_t* prep_shares, uint8_t* jr_seeds, uint8_t* out_shares,
                       int32_t* status);
/* Both aggregators' prep_shares_to_prep + prep_next (mastic.py:320-377) for
 * the last mastic_prep_init of agg_id 0 and of agg_id 1 on this ctx (same
 * reports and agg param, e.g. a heavy-hitters sweep driving both aggregators
 * on one GPU): the prep shares never leave HBM.  accept_out[i] (n, may be
 * NULL) = 1 iff the eval proofs agree, the FLP decides true (weight check),
 * neither query aborted and both joint-rand seeds equal the prep message;
 * decide_out[i] (n, may be NULL) = the MASTIC_DECIDE_* code. */
int mastic_decide_results(mastic_ctx* ctx, const uint8_t* app_ctx, size_t ctx_len, uint8_t* accept_out,
                          uint8_t* decide_out);
/* Fold the out shares of the last prep_init for agg_id over the reports whose
 * valid[i] != 0 (valid == NULL: all) into agg_share
 * (len(prefixes)*(1+output_len)*field_bytes, encode_vec). */
int mastic_aggregate(mastic_ctx* ctx, int agg_id, const uint8_t* valid, uint8_t* agg_share);
/* mastic_aggregate into a caller-owned DEVICE buffer of the ctx's GPU (same
 * layout), e.g. the send buffer of an RCCL all-gather: the share never
 * leaves HBM.  caller_stream is the hipStream_t whose queued work last
 * touched the buffer (e.g. the stream it was allocated or zero-filled on;
 * NULL = the null stream): the fold is ordered after that work by an event.
 * Returns when the buffer is written. */
int mastic_aggregate_device_on_stream(mastic_ctx* ctx, int agg_id, const uint8_t* valid, void* dev_agg_share,
                                      void* caller_stream);
/* Multi-GPU merge (Mastic.merge, mastic.py:390-397) of n_shares agg shares
 * of n_elems elements each, all in DEVICE memory of the ctx's GPU (e.g. the
 * output of an RCCL all-gather): dev_out[e] = sum_s dev_shares[s][e] mod p.
 * Elements are in encode_vec byte order.  producer_stream is the hipStream_t
 * the shares were written on (NULL = the null stream): the fold is ordered
 * after that stream's queued work by an event.  Returns when dev_out is
 * written. */
int mastic_fold_shares(mastic_ctx* ctx, const void* dev_shares, size_t n_shares, size_t n_elems, void* dev_out,
                       void* producer_stream);
/* ---- multi-GPU aggregation over a library-owned RCCL communicator ------
 * One process per GPU, reports split over the ranks.  The
 * only exchange is the per-prefix agg share: an RCCL all-gather over xGMI,
 * then the GF(p) fold on the GPU (RCCL's integer sum is not field addition).
 * Replaces Mastic.merge (mastic.py:390-397) of the ranks' agg shares.
 * Rank 0 calls mastic_comm_unique_id and hands the id to every rank by any
 * channel it likes (a file, a socket, a launcher's store); each rank then
 * calls mastic_comm_init on its ctx (collective: returns when all nranks
 * ranks have joined).  A ctx without a communicator behaves as world 1.
 * librccl is loaded on the first call of this group (MASTIC_ENODEV if it
 * cannot be).
 *
 * Failure model of every collective call below (mastic_allgather_fold,
 * mastic_merge_host, mastic_aggregate_merged): each rank first does its local
 * work (argument checks, staging allocations, the local fold), then all ranks
 * exchange a status record; a rank whose local work failed still takes part.
 * If any rank failed, no share bytes move: a failing rank returns its own
 * error, every other rank the code of the lowest failing rank; calls that
 * disagree on the entry point, n_local or n_elems return MASTIC_EINVAL on
 * every rank.  Every wait on the communicator (init included) is bounded by
 * the ctx's timeout, which starts once this rank's own queued work is done
 * (so a long prep_init ahead of a merge does not count against it): a peer
 * that never joins yields MASTIC_ETIMEDOUT.  A
 * timed-out init is abandoned (the ctx stays world 1; RCCL's pending init
 * stays on a library thread, which releases the communicator if the peers
 * ever arrive); a timed-out collective aborts the communicator, and later
 * collective calls fail with MASTIC_EHIP (never a silent world-1 merge) until
 * mastic_comm_destroy and a new mastic_comm_init.  Host output buffers
 * (host_out, agg_out) are written only after the bounded wait succeeded; on
 * any error they are left untouched.  Test hook: the environment variable
 * MASTIC_RCCL_LIB names a library to bind instead of librccl (no fallback);
 * tests/host/fake_rccl.cpp is a shared-memory stand-in that lets several
 * processes on one GPU form a communicator. */
#define MASTIC_COMM_ID_BYTES 128
#define MASTIC_COMM_TIMEOUT_MS 120000 /* mastic_comm_init's bound on every communicator wait */
int mastic_comm_unique_id(uint8_t id_out[MASTIC_COMM_ID_BYTES]);
int mastic_comm_init(mastic_ctx* ctx, int nranks, int rank, const uint8_t id[MASTIC_COMM_ID_BYTES]);
/* mastic_comm_init with the bound (ms, > 0; <= 0: MASTIC_COMM_TIMEOUT_MS) on
 * the init itself and on every later wait on this communicator. */
int mastic_comm_init_timeout(mastic_ctx* ctx, int nranks, int rank, const uint8_t id[MASTIC_COMM_ID_BYTES],
                             int timeout_ms);
/* Number of ranks / this rank of the ctx's communicator (1 / 0 without one). */
int mastic_comm_info(const mastic_ctx* ctx, int* nranks, int* rank);
int mastic_comm_destroy(mastic_ctx* ctx);
/* dev_out[e] = sum over every rank r and local share s of
 * dev_local_r[s][e] mod p: each rank passes n_local shares of n_elems
 * elements (encode_vec order) in DEVICE memory, all ranks the same counts.
 * The all-gather and the fold run on the ctx's stream, ordered after
 * caller_stream's queued work (NULL = the null stream) by an event.
 * Collective; returns when dev_out is written. */
int mastic_allgather_fold(mastic_ctx* ctx, const void* dev_local, size_t n_local, size_t n_elems, void* dev_out,
                          void* caller_stream);
/* mastic_allgather_fold on HOST buffers (shares a driver holds in host
 * memory, e.g. decoded agg shares): host_local n_local x n_elems elements in,
 * host_out n_elems elements out; staged through the ctx's device buffers.
 * Collective. */
int mastic_merge_host(mastic_ctx* ctx, const uint8_t* host_local, size_t n_local, size_t n_elems, uint8_t* host_out);
/* The whole agg_update + merge of a sharded job in HBM: each selected
 * aggregator's (agg_mask bit a = agg_id a) out shares of its last prep_init
 * are folded over the reports with valid[i] != 0 (NULL: all) on this GPU,
 * all-gathered across the communicator's ranks, and summed mod p; agg_out
 * (host, n_elems * field_bytes) receives the sum over ranks and over the
 * selected aggregators.  n_elems = len(prefixes) * (1 + output_len) must
 * match that prep_init.  A rank that ran no prep_init for this agg param
 * (no reports on it) adds MASTIC_MERGE_ZEROS and contributes agg_init's
 * zeros for the selected aggregators.  agg_mask 1 or 2: that aggregator's
 * job-wide agg share; 3: the collector's merge of both (the heavy-hitters
 * sweep's per-level total).  Collective: every rank passes the same
 * aggregators and n_elems. */
#define MASTIC_MERGE_ZEROS 4u
int mastic_aggregate_merged(mastic_ctx* ctx, uint32_t agg_mask, const uint8_t* valid, size_t n_elems,
                            uint8_t* agg_out);
/* VIDPF-proof aggregation mode (draft-mouris-cfrg-mastic.md, "Plain
 * Heavy-Hitters with VIDPF-Proof Aggregation"; no poc code or wire format in
 * the reference): Merkle tree over the eval proofs of the last prep_init of
 * agg_id.  Leaves = the n eval proofs (32 B each, report order); a node of two
 * children = XofTurboShake128(b"", dst(app_ctx, 12), left || right).next(32);
 * the last node of an odd level is promoted unchanged.  nodes_out receives
 * all levels, leaves first, 32 B per node; n_nodes must equal
 * n + ceil(n/2) + ... + 1 (0 for n = 0).  Both aggregators' roots are equal iff
 * every report's eval proofs agree (mastic.py:340). */
int mastic_proof_tree(mastic_ctx* ctx, int agg_id, const uint8_t* app_ctx, size_t ctx_len, uint8_t* nodes_out,
                      size_t n_nodes);
/* Frontier cache for level sweeps (the reference's
 * examples.py:37-91 re-evaluates the whole tree at every level).  on = 1
 * enables it, 0 disables it and frees its buffers, -1 leaves it unchanged.
 * With it on, prep_init keeps per report the two binder sponges' states
 * (400 B) plus the last level's seeds, control bits and convert seeds; a
 * later prep_init for the same reports, agg_id, verify key and ctx whose tree
 * is the cached tree plus one level (the sweep with no candidate path pruned
 * away) recomputes its parents' payloads from their convert seeds, evaluates
 * only that level and resumes the sponges from the cached states (the binder messages
 * are BFS-ordered, so the cached ones are prefixes of the new ones).  Results
 * are identical either way.  *last_hit (if not NULL) = 1 when the last
 * prep_init took the cached path. */
int mastic_set_frontier_cache(mastic_ctx* ctx, int on, int* last_hit);
/* Measurement schedule: on = 1 makes every binder-sponge launch run alone
 * (the level kernels wait for it instead of running beside it), so the
 * sponge kernels' and the level kernel's own rates can be timed
 * (mastic_last_timing3); 0 restores the overlapped schedule, -1 only queries.
 * Results are identical either way.  Returns the previous setting (0 / 1) or
 * MASTIC_EINVAL. */
int mastic_set_serial_sponges(mastic_ctx* ctx, int on);
/* Wait for all enqueued work of the ctx. */
int mastic_synchronize(mastic_ctx* ctx);
/* The library's MASTIC_ABI_VERSION (a caller built against another header
 * version must not bind it). */
int mastic_abi_version(void);
/* Result-preserving test hooks of one ctx (tests only; the library reads no
 * environment variable that changes computation).  force_slow_blk >= 0: the
 * level kernel's speculative payload path hands over to the exact
 * rejection-sampling stream (vidpf.py:352-364 next_vec) at this convert block,
 * which random data reaches with probability ~2^-32 per candidate; -1 off.
 * fail_allocs: the next that many result-buffer / frontier-cache-slot
 * allocations fail as if HBM were exhausted, driving the recovery path (wait
 * for the ctx's streams, free retired buffers and the work arena, retry); a
 * collective call's staging allocations fail the same way (that call then
 * returns MASTIC_ENOMEM on every rank, after the agreement round).
 * Outputs are identical either way.  Returns the number of injected failures
 * the previous setting still had pending (>= 0), or MASTIC_EINVAL. */
int mastic_set_test_hooks(mastic_ctx* ctx, int force_slow_blk, int fail_allocs);
/* Test hook: the next mastic_prep_init that records empty timing marks on
 * the ctx's binder-sponge stream (level 0 of a call, a frontier-cache hit)
 * first queues there a kernel that idles delay_us microseconds (0..10^7), so
 * those marks complete late while nothing on the main stream waits for them
 * (mastic_last_timing* must wait for the marks themselves).  Results are
 * unaffected. */
int mastic_set_test_sponge_delay(mastic_ctx* ctx, int delay_us);

/* One-shot host-buffer form of upload + prep_init + prep_result. */
int mastic_prep_init_batch(mastic_ctx* ctx, const uint8_t* verify_key, size_t verify_key_len,
                           const uint8_t* app_ctx, size_t ctx_len, int agg_id, const uint8_t* enc_agg_param, size_t agg_param_len, size_t n,
                           const uint8_t* nonces, const uint8_t* public_shares, const uint8_t* input_shares,
                           uint8_t* prep_shares_out, uint8_t* jr_seeds_out, uint8_t* out_shares_out,
                           int32_t* status_out);

/* prep_shares_to_prep for n report pairs.  prep_msgs_out n*32 (joint-rand
 * confirmation seed; untouched when the circuit has no joint randomness) may
 * be NULL.  valid_out[i]: MASTIC_DECIDE_OK when both checks pass (eval proofs
 * equal and, with the weight check, the FLP decides true);
 * MASTIC_DECIDE_VIDPF_FAIL / MASTIC_DECIDE_FLP_FAIL mirror the reference's
 * 'VIDPF verification failed' / 'FLP verification failed' exceptions. */
#define MASTIC_DECIDE_VIDPF_FAIL 0
#define MASTIC_DECIDE_OK 1
#define MASTIC_DECIDE_FLP_FAIL 2
int mastic_decide_batch(mastic_ctx* ctx, const uint8_t* app_ctx, size_t ctx_len, const uint8_t* enc_agg_param,
                        size_t agg_param_len, size_t n, const uint8_t* prep_shares0, const uint8_t* prep_shares1,
                        uint8_t* prep_msgs_out, uint8_t* valid_out);

/* One-shot client shard of n reports into host buffers. */
int mastic_shard_batch(mastic_ctx* ctx, const uint8_t* app_ctx, size_t ctx_len, size_t n, const uint8_t* alphas,
                       const uint8_t* betas, const uint8_t* nonces, const uint8_t* rands, uint8_t* public_shares_out,
                       uint8_t* input_shares0_out, uint8_t* input_shares1_out);

/* ---- measurement hooks (bench) --------------------------------------- */
/* Device time (ms) of the VIDPF level-eval (AES) kernels and of the
 * binder-absorb kernels during the last prep_init, measured with HIP events on
 * the streams the kernels run on; also their launch counts.  Timing is kept
 * per aggregator: "last" is the aggregator of the latest prep_init or
 * mastic_prep_result call, so both aggregators' prep_init may be queued before
 * either result is fetched. */
int mastic_last_timing(mastic_ctx* ctx, double* eval_ms, int* eval_launches, double* absorb_ms,
                       int* absorb_launches, double* total_ms);
/* HBM work-buffer bytes one report needs during prep_init with this agg
 * param (prep_init processes reports in chunks of budget / this). */
int mastic_work_bytes(mastic_ctx* ctx, const uint8_t* enc_agg_param, size_t agg_param_len, uint64_t* per_report);
/* The same split three ways: VIDPF AES level kernels, node-proof (Keccak)
 * level kernels, binder-sponge kernels (ms summed over launches). */
int mastic_last_timing3(mastic_ctx* ctx, double* aes_ms, int* aes_launches, double* proof_ms, int* proof_launches,
                        double* absorb_ms, int* absorb_launches, double* total_ms);
/* Tree statistics of an encoded agg param: nodes evaluated per report,
 * interior nodes, max nodes on one level. */
int mastic_tree_stats(mastic_ctx* ctx, const uint8_t* enc_agg_param, size_t agg_param_len, uint64_t* nodes,
                      uint64_t* interior, uint64_t* max_level_nodes);

#ifdef __cplusplus
}
#endif
#endif
