// The agreement round of the library's collective calls (mastic_hip.hip
// comm_agree; include/mastic_hip.h, "failure model"): one 32-byte record per
// rank, all-gathered, and the decision every rank takes from the same
// gathered array.  Free of HIP and RCCL, so the multi-rank decision runs on
// the host in tests/host/comm_agree_host.cpp under ASan/UBSan.
#pragma once
#include <stddef.h>
#include <stdint.h>

// One rank's record.
struct CommStatus {
    int32_t rc;        // 0 = this rank's local work succeeded, else its MASTIC_E* code
    uint32_t op;       // entry point (CommOp)
    uint64_t n_local;  // shares per rank
    uint64_t n_elems;  // elements per share
    uint32_t magic;
    uint32_t pad;
};
static_assert(sizeof(CommStatus) == 32, "CommStatus layout");
constexpr uint32_t COMM_MAGIC = 0x4d415354u;
enum CommOp : uint32_t { COMM_ALLGATHER_FOLD = 1, COMM_MERGE_HOST = 2, COMM_AGGREGATE_MERGED = 3 };

inline const char* comm_op_name(uint32_t op) {
    return op == COMM_ALLGATHER_FOLD     ? "mastic_allgather_fold"
           : op == COMM_MERGE_HOST       ? "mastic_merge_host"
           : op == COMM_AGGREGATE_MERGED ? "mastic_aggregate_merged"
                                         : "?";
}

// What the gathered records say, identical on every rank.
struct CommVerdict {
    int first_bad = -1;  // lowest rank whose local work failed (its rc is the verdict's code)
    int mismatch = -1;   // lowest rank whose record disagrees with this call (entry point, geometry, magic)
    int32_t bad_rc = 0;
};

inline CommVerdict comm_decide(const CommStatus* all, int nranks, uint32_t op, uint64_t n_local, uint64_t n_elems) {
    CommVerdict v;
    for (int r = 0; r < nranks; r++) {
        const CommStatus& s = all[r];
        if (s.magic != COMM_MAGIC) {  // not a record: its rc means nothing
            if (v.mismatch < 0) v.mismatch = r;
        } else if (s.rc != 0) {
            // a failure counts whatever call the rank made, so every rank
            // (the odd one out of a disagreement too) reports the same code
            if (v.first_bad < 0) {
                v.first_bad = r;
                v.bad_rc = s.rc;
            }
        } else if (s.op != op || s.n_local != n_local || s.n_elems != n_elems) {
            if (v.mismatch < 0) v.mismatch = r;
        }
    }
    return v;
}

// The code this rank returns: its own failure first, else the lowest failing
// rank's code, else EINVAL (einval) for a call the ranks disagree on, else 0
// (every rank ready: the data exchange may run).
inline int comm_rank_result(const CommVerdict& v, int local_rc, int einval) {
    if (local_rc) return local_rc;
    if (v.first_bad >= 0) return v.bad_rc;
    if (v.mismatch >= 0) return einval;
    return 0;
}
