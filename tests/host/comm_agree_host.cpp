// Host harness for the collective calls' agreement round
// (draft-mouris-cfrg-mastic_amd/csrc/comm_agree.hpp, used by mastic_hip.hip
// comm_agree): N simulated ranks each contribute a status record, the
// "all-gather" is the array of all records in rank order, and every rank
// derives its return code from that same array.  Prints one line per case:
//   case <name> codes=<rank 0 code>,<rank 1 code>,...
// Run under ASan/UBSan by tests/test_comm_agree_host.py.
#include <cstdio>
#include <string>
#include <vector>

#include "../../draft-mouris-cfrg-mastic_amd/csrc/comm_agree.hpp"

static constexpr int EINVAL_ = -22;

struct Call {
    int rc;
    uint32_t op;
    uint64_t n_local, n_elems;
    uint32_t magic = COMM_MAGIC;
};

static void run(const char* name, const std::vector<Call>& calls) {
    std::vector<CommStatus> gathered;
    for (const Call& k : calls) gathered.push_back(CommStatus{k.rc, k.op, k.n_local, k.n_elems, k.magic, 0});
    std::string codes;
    for (size_t r = 0; r < calls.size(); r++) {
        // each rank decides with ITS OWN call's op and geometry
        const CommVerdict v = comm_decide(gathered.data(), (int)gathered.size(), calls[r].op, calls[r].n_local,
                                          calls[r].n_elems);
        const int rc = comm_rank_result(v, calls[r].rc, EINVAL_);
        codes += (r ? "," : "") + std::to_string(rc);
    }
    printf("case %-24s codes=%s\n", name, codes.c_str());
}

int main() {
    const uint32_t A = COMM_AGGREGATE_MERGED, F = COMM_ALLGATHER_FOLD;
    std::vector<Call> ok(8, Call{0, A, 2, 728});
    run("all ready", ok);
    {
        auto c = ok;
        c[5].rc = -12;  // rank 5 could not allocate its staging buffer
        run("enomem on rank 5", c);
    }
    {
        auto c = ok;
        c[2].rc = -22;
        c[6].rc = -12;
        run("einval 2, enomem 6", c);
    }
    {
        auto c = ok;
        c[3].n_elems = 730;  // rank 3 merges another level's shares
        run("geometry on rank 3", c);
    }
    {
        auto c = ok;
        c[7].op = F;  // rank 7 entered another collective
        run("entry point on rank 7", c);
    }
    {
        auto c = ok;
        c[1].magic = 0;  // a corrupted record
        run("bad record on rank 1", c);
    }
    {
        auto c = ok;
        c[4].n_local = 1;
        c[6].rc = -5;  // a failure outranks a disagreement
        run("failure and mismatch", c);
    }
    {
        std::vector<Call> one{Call{0, F, 3, 301}};
        run("world 1", one);
        one[0].rc = -12;
        run("world 1 enomem", one);
    }
    {
        std::vector<Call> z(4, Call{0, A, 2, 0});  // every rank has an empty candidate list
        run("zero elements", z);
    }
    printf("comm_agree_host: OK\n");
    return 0;
}
