// Test infrastructure only: a stand-in for the eight RCCL entry points
// libmastic_hip binds (mastic_hip.hip, RcclApi), loaded through the
// MASTIC_RCCL_LIB test hook, so that several processes sharing ONE GPU can
// form a communicator.  RCCL itself refuses two ranks on one device
// ("Duplicate GPU detected"), and the builder has no multi-GPU box, so this is
// how the library's N-rank collective code -- the agreement round, the
// failure propagation, the bounded waits and the abort, the all-gather + GF(p)
// fold -- runs on a real GPU at N > 1 (tests/test_gpu_comm_nrank.py).
//
// Transport: POSIX shared memory between the ranks' processes.  The
// communicator behaves like a NON-BLOCKING RCCL communicator: ncclAllGather
// returns ncclInProgress and a worker thread (1) copies the send buffer to
// pinned host memory and waits for it, (2) publishes the bytes and waits for
// every rank's, (3) gathers them and queues the copy into the receive buffer on
// the caller's stream, then reports ncclSuccess through ncclCommGetAsyncError.
// A missing peer leaves the call in progress until the caller gives up and
// calls ncclCommAbort, which stops the worker.  (An earlier form ran step 2 as
// a stream host function; with three ranks one rank's stream then stayed
// busy after its host function had returned.)  Only ncclUint8 is used by the
// library; every count is in bytes.  FAKE_RCCL_TRACE=1 logs each step.
#include <hip/hip_runtime_api.h>
#include <rccl/rccl.h>

#include <atomic>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fcntl.h>
#include <random>
#include <sys/mman.h>
#include <thread>
#include <unistd.h>

namespace {
constexpr int MAX_RANKS = 16;
constexpr size_t SLOT_BYTES = size_t(8) << 20;  // largest all-gather contribution per rank
constexpr uint32_t ID_MAGIC = 0x46524343u;      // "FRCC"

struct Shared {
    std::atomic<int> joined;
    std::atomic<int> mapped;
    std::atomic<uint64_t> arrived[MAX_RANKS];   // last generation whose bytes rank r published
    std::atomic<uint64_t> departed[MAX_RANKS];  // last generation rank r has gathered
};

struct IdLayout {
    uint32_t magic;
    char name[64];
};
static_assert(sizeof(IdLayout) <= sizeof(ncclUniqueId), "id layout");

size_t shm_bytes(int nranks) { return sizeof(Shared) + (size_t)nranks * SLOT_BYTES; }

bool trace() {
    static const bool on = [] {
        const char* e = getenv("FAKE_RCCL_TRACE");
        return e && *e == '1';
    }();
    return on;
}
}  // namespace

struct ncclComm {
    int nranks = 0, rank = 0, device = 0;
    Shared* sh = nullptr;
    uint8_t* slots = nullptr;
    uint8_t* pin_send = nullptr;  // pinned host staging
    uint8_t* pin_recv = nullptr;
    uint64_t gen = 0;
    std::atomic<bool> aborted{false};
    std::atomic<int> state{ncclSuccess};  // of the last all-gather (ncclInProgress while its worker runs)
    std::thread worker;
};

namespace {
void say(const ncclComm* c, uint64_t g, const char* what) {
    if (trace()) fprintf(stderr, "[fake rccl %d] gen %llu: %s\n", c->rank, (unsigned long long)g, what);
}

// Wait until pred() holds or the communicator is aborted (returns false then).
template <class P>
bool wait_for(ncclComm* c, P pred) {
    for (int spin = 0; !pred(); spin++) {
        if (c->aborted.load(std::memory_order_acquire)) return false;
        if (spin < 1000)
            std::this_thread::yield();
        else
            std::this_thread::sleep_for(std::chrono::microseconds(50));
    }
    return true;
}

// One all-gather, on the communicator's worker thread.
void gather(ncclComm* c, uint64_t g, const void* send, void* recv, size_t bytes, hipStream_t stream) {
    Shared* sh = c->sh;
    ncclResult_t r = ncclSystemError;
    if (hipSetDevice(c->device) == hipSuccess &&
        hipMemcpyAsync(c->pin_send, send, bytes, hipMemcpyDeviceToHost, stream) == hipSuccess &&
        hipStreamSynchronize(stream) == hipSuccess) {
        // every rank has gathered generation g - 1, so its slot may be reused
        bool ok = wait_for(c, [&] {
            for (int q = 0; q < c->nranks; q++)
                if (sh->departed[q].load(std::memory_order_acquire) + 1 < g) return false;
            return true;
        });
        if (ok) {
            std::memcpy(c->slots + (size_t)c->rank * SLOT_BYTES, c->pin_send, bytes);
            sh->arrived[c->rank].store(g, std::memory_order_release);
            say(c, g, "published");
            ok = wait_for(c, [&] {
                for (int q = 0; q < c->nranks; q++)
                    if (sh->arrived[q].load(std::memory_order_acquire) < g) return false;
                return true;
            });
        }
        if (ok) {
            for (int q = 0; q < c->nranks; q++)
                std::memcpy(c->pin_recv + (size_t)q * bytes, c->slots + (size_t)q * SLOT_BYTES, bytes);
            sh->departed[c->rank].store(g, std::memory_order_release);
            // pin_recv is rewritten only by the next all-gather, which first
            // synchronizes the stream, i.e. this copy
            r = hipMemcpyAsync(recv, c->pin_recv, bytes * (size_t)c->nranks, hipMemcpyHostToDevice, stream) ==
                        hipSuccess
                    ? ncclSuccess
                    : ncclSystemError;
            say(c, g, "gathered");
        } else {
            r = ncclRemoteError;
            say(c, g, "aborted");
        }
    }
    c->state.store(r, std::memory_order_release);
}

void join_worker(ncclComm* c) {
    if (c->worker.joinable()) c->worker.join();
}
}  // namespace

extern "C" {

const char* ncclGetErrorString(ncclResult_t r) {
    switch (r) {
        case ncclSuccess: return "no error (fake RCCL)";
        case ncclInvalidArgument: return "invalid argument (fake RCCL)";
        case ncclInvalidUsage: return "invalid usage (fake RCCL)";
        case ncclSystemError: return "system error (fake RCCL)";
        case ncclRemoteError: return "aborted while waiting for a peer (fake RCCL)";
        default: return "error (fake RCCL)";
    }
}

ncclResult_t ncclGetUniqueId(ncclUniqueId* id) {
    if (!id) return ncclInvalidArgument;
    std::memset(id, 0, sizeof(*id));
    IdLayout l{};
    l.magic = ID_MAGIC;
    std::random_device rd;
    snprintf(l.name, sizeof l.name, "/mastic_fake_rccl_%d_%08x%08x", (int)getpid(), rd(), rd());
    std::memcpy(id, &l, sizeof l);
    return ncclSuccess;
}

// Blocks until every rank has joined, as RCCL's bootstrap does.
ncclResult_t ncclCommInitRank(ncclComm_t* out, int nranks, ncclUniqueId id, int rank) {
    IdLayout l;
    std::memcpy(&l, &id, sizeof l);
    if (!out || l.magic != ID_MAGIC || nranks < 1 || nranks > MAX_RANKS || rank < 0 || rank >= nranks)
        return ncclInvalidArgument;
    int device = 0;
    if (hipGetDevice(&device) != hipSuccess) return ncclSystemError;
    const int fd = shm_open(l.name, O_CREAT | O_RDWR, 0600);
    if (fd < 0) return ncclSystemError;
    const size_t bytes = shm_bytes(nranks);
    if (ftruncate(fd, (off_t)bytes) != 0) {
        close(fd);
        return ncclSystemError;
    }
    void* p = mmap(nullptr, bytes, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
    close(fd);
    if (p == MAP_FAILED) return ncclSystemError;
    ncclComm* c = new ncclComm;
    c->nranks = nranks;
    c->rank = rank;
    c->device = device;
    c->sh = (Shared*)p;  // zero-filled by ftruncate: counters start at 0
    c->slots = (uint8_t*)p + sizeof(Shared);
    if (hipHostMalloc((void**)&c->pin_send, SLOT_BYTES, hipHostMallocDefault) != hipSuccess ||
        hipHostMalloc((void**)&c->pin_recv, SLOT_BYTES * nranks, hipHostMallocDefault) != hipSuccess) {
        munmap(p, bytes);
        delete c;
        return ncclSystemError;
    }
    c->sh->joined.fetch_add(1);
    while (c->sh->joined.load() < nranks) std::this_thread::sleep_for(std::chrono::microseconds(200));
    // the last rank to map the segment unlinks its name: nothing is left in /dev/shm
    if (c->sh->mapped.fetch_add(1) + 1 == nranks) shm_unlink(l.name);
    *out = c;
    return ncclSuccess;
}

ncclResult_t ncclAllGather(const void* send, void* recv, size_t count, ncclDataType_t type, ncclComm_t c,
                           hipStream_t stream) {
    if (!c || type != ncclUint8 || count > SLOT_BYTES || (count && (!send || !recv))) return ncclInvalidArgument;
    if (c->aborted.load() || c->state.load() == ncclInProgress) return ncclInvalidUsage;
    if (count == 0) return ncclSuccess;
    join_worker(c);
    const uint64_t g = ++c->gen;
    say(c, g, "queued");
    c->state.store(ncclInProgress);
    c->worker = std::thread(gather, c, g, send, recv, count, stream);
    return ncclInProgress;
}

ncclResult_t ncclCommGetAsyncError(ncclComm_t c, ncclResult_t* st) {
    if (!c || !st) return ncclInvalidArgument;
    *st = (ncclResult_t)c->state.load(std::memory_order_acquire);
    return ncclSuccess;
}

// Local release: an all-gather waiting for a peer stops (its receive buffer
// is not written); peers are not told.  The shared segment and the pinned
// buffers stay mapped (a test-only leak per aborted communicator): the
// caller's stream may still hold copies from them.
ncclResult_t ncclCommAbort(ncclComm_t c) {
    if (!c) return ncclSuccess;
    c->aborted.store(true, std::memory_order_release);
    join_worker(c);
    return ncclSuccess;
}

ncclResult_t ncclCommFinalize(ncclComm_t c) { return c ? ncclSuccess : ncclInvalidArgument; }

// After the caller has waited for its stream (mastic_comm_destroy does).
ncclResult_t ncclCommDestroy(ncclComm_t c) {
    if (!c) return ncclInvalidArgument;
    join_worker(c);
    munmap(c->sh, shm_bytes(c->nranks));
    (void)hipHostFree(c->pin_send);
    (void)hipHostFree(c->pin_recv);
    delete c;
    return ncclSuccess;
}

}  // extern "C"
