// lpc_comm.hpp -- the per-iteration exchange of a ray-sharded trace.
//
// The reference traces all rays in one process and takes two global decisions
// per iteration: stop when the power left in the scene falls below
// (1 - trace_until_dissipated) * input power, or when no ray is left
// (/root/reference/iterative_tracer.py:372-391).  With the rays sharded over
// one process per GPU those decisions need the sums over all ranks: a handful
// of doubles per iteration, on the critical path between two iterations.
//
// lpc_trace_run's loop calls an all-reduce hook (lpc_allreduce_fn) for them.
// The library's own hook is a host all-reduce over POSIX shared memory for the
// ranks of one node (the driver's 1/2/4/8-GPU runs): each rank publishes its
// values in its own cache-line-aligned slot with a sequence number and sums
// all slots in rank order, so every rank computes the identical bits and takes
// the identical decision.  The counters it reduces are already on the host
// (the mapped copy k_stage_move publishes), so no device round trip is added;
// ~1 us per exchange against ~20-60 us for a torch.distributed call.  Any
// other transport (gloo in the CPU tests, RCCL) plugs in through the same hook.
#pragma once

#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <chrono>
#include <cstdint>
#include <cstring>
#include <string>
#include <thread>

namespace lpcc {

const uint32_t kMagic = 0x4c504353u;      // "LPCS"
const int32_t kCap = 8192;                // doubles per exchange chunk
const double kTimeoutS = 300.0;           // a peer that never arrives: error, not a hang

struct alignas(64) ShmHdr {
    volatile uint32_t magic;
    int32_t world;
    int32_t cap;
    uint32_t pad[13];
};

struct alignas(64) ShmSlot {
    volatile uint64_t seq;                // last exchange this rank published
    volatile uint64_t abort;              // != 0: this rank gave up; its peers fail fast
    uint64_t pad[6];
    double v[2][kCap];                    // double-buffered by exchange parity
};

struct ShmComm {
    std::string name;
    int32_t rank = 0, world = 1;
    bool owner = false, unlinked = false;
    size_t bytes = 0;
    void *base = nullptr;
    uint64_t seq = 0;
    bool failed = false;                  // an exchange failed: the ranks' sequence numbers are
                                          // out of step, every later exchange is an error
    std::string err;
    ShmHdr *hdr() const { return (ShmHdr *)base; }
    ShmSlot *slot(int r) const { return (ShmSlot *)((char *)base + sizeof(ShmHdr)) + r; }
};

inline size_t shm_bytes(int32_t world) { return sizeof(ShmHdr) + (size_t)world * sizeof(ShmSlot); }

inline double now_s()
{
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

// rank 0 (create != 0) creates and initialises the segment; the others wait
// for it to appear with the right size and magic.
inline int shm_open_comm(const char *name, int32_t rank, int32_t world, int create, ShmComm **out,
                         std::string *err)
{
    if (!name || !out || world < 1 || rank < 0 || rank >= world) { *err = "shm comm: bad argument"; return -1; }
    ShmComm *c = new ShmComm();
    c->name = name[0] == '/' ? name : std::string("/") + name;
    c->rank = rank;
    c->world = world;
    c->owner = create != 0;
    c->bytes = shm_bytes(world);
    int fd = -1;
    const double t0 = now_s();
    if (c->owner) {
        fd = shm_open(c->name.c_str(), O_CREAT | O_EXCL | O_RDWR, 0600);
        if (fd < 0 || ftruncate(fd, (off_t)c->bytes) != 0) {
            *err = "shm comm: cannot create " + c->name + ": " + strerror(errno);
            if (fd >= 0) { close(fd); shm_unlink(c->name.c_str()); }
            delete c;
            return -1;
        }
    } else {
        for (;;) {
            fd = shm_open(c->name.c_str(), O_RDWR, 0600);
            if (fd >= 0) {
                struct stat st;
                if (fstat(fd, &st) == 0 && (size_t)st.st_size >= c->bytes) break;
                close(fd);
                fd = -1;
            }
            if (now_s() - t0 > kTimeoutS) { *err = "shm comm: " + c->name + " never appeared"; delete c; return -1; }
            std::this_thread::sleep_for(std::chrono::milliseconds(1));
        }
    }
    c->base = mmap(nullptr, c->bytes, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
    close(fd);
    if (c->base == MAP_FAILED) {
        *err = "shm comm: mmap failed";
        if (c->owner) shm_unlink(c->name.c_str());
        delete c;
        return -1;
    }
    if (c->owner) {
        memset(c->base, 0, c->bytes);
        c->hdr()->world = world;
        c->hdr()->cap = kCap;
        __atomic_store_n(&c->hdr()->magic, kMagic, __ATOMIC_RELEASE);
    } else {
        while (__atomic_load_n(&c->hdr()->magic, __ATOMIC_ACQUIRE) != kMagic) {
            if (now_s() - t0 > kTimeoutS) { *err = "shm comm: segment never initialised"; munmap(c->base, c->bytes); delete c; return -1; }
            std::this_thread::sleep_for(std::chrono::milliseconds(1));
        }
        if (c->hdr()->world != world) { *err = "shm comm: world size mismatch"; munmap(c->base, c->bytes); delete c; return -1; }
    }
    *out = c;
    return 0;
}

// Give up on the comm: every later exchange on it fails, and so do the peers'
// waits (they see this rank's abort word instead of spinning to the timeout) and
// the peers' current exchange if they were past their wait (the abort words are
// checked again before the sum).
inline void shm_abort(ShmComm *c, const std::string &why)
{
    if (!c) return;
    if (!c->failed) c->err = why;
    c->failed = true;
    if (c->base) __atomic_store_n(&c->slot(c->rank)->abort, (uint64_t)1, __ATOMIC_RELEASE);
}

// In-place sum over all ranks, identical bits on every rank (rank-order sums).
// Exchange s writes buffer s & 1 of this rank's slot: a rank starts exchange s
// only after every rank published s - 1, i.e. finished reading exchange s - 2,
// the last user of that buffer.  A timeout or a peer's abort word breaks the
// comm for good (shm_abort): after a failed exchange the ranks no longer agree
// on which call pairs with which, so no later sum could be trusted.
inline int shm_allreduce(ShmComm *c, double *vals, int32_t n)
{
    if (!c || (n > 0 && !vals) || n < 0) return -1;
    if (c->failed) {
        if (c->err.empty()) c->err = "shm comm: broken by an earlier failed exchange";
        return -1;
    }
    if (c->world == 1) return 0;
    for (int32_t off = 0; off < n || (n == 0 && off == 0); off += kCap) {
        const int32_t m = n - off < kCap ? n - off : kCap;
        const uint64_t s = ++c->seq;
        const int b = (int)(s & 1u);
        ShmSlot *me = c->slot(c->rank);
        if (m > 0) memcpy(me->v[b], vals + off, (size_t)m * 8);
        __atomic_store_n(&me->seq, s, __ATOMIC_RELEASE);
        const double t0 = now_s();
        for (int r = 0; r < c->world; ++r) {
            uint64_t spins = 0;
            while (__atomic_load_n(&c->slot(r)->seq, __ATOMIC_ACQUIRE) < s) {
                if (__atomic_load_n(&c->slot(r)->abort, __ATOMIC_ACQUIRE) != 0) {
                    shm_abort(c, "shm comm: rank " + std::to_string(r) + " aborted before exchange " +
                                     std::to_string(s));
                    return -1;
                }
                if ((++spins & 1023u) == 0u && now_s() - t0 > kTimeoutS) {
                    shm_abort(c, "shm comm: rank " + std::to_string(r) + " did not reach exchange " +
                                     std::to_string(s));
                    return -1;
                }
                __builtin_ia32_pause();
            }
        }
        // a peer that published this exchange and then gave up (its own wait
        // timed out): its values may be from an exchange the others never paired
        // with it, so no rank sums them
        for (int r = 0; r < c->world; ++r)
            if (__atomic_load_n(&c->slot(r)->abort, __ATOMIC_ACQUIRE) != 0) {
                shm_abort(c, "shm comm: rank " + std::to_string(r) + " aborted during exchange " + std::to_string(s));
                return -1;
            }
        for (int32_t i = 0; i < m; ++i) {
            double acc = 0.0;
            for (int r = 0; r < c->world; ++r) acc += c->slot(r)->v[b][i];
            vals[off + i] = acc;
        }
        if (n == 0) break;
    }
    return 0;
}

inline void shm_unlink_comm(ShmComm *c)
{
    if (c && c->owner && !c->unlinked) { shm_unlink(c->name.c_str()); c->unlinked = true; }
}

inline void shm_close_comm(ShmComm *c)
{
    if (!c) return;
    shm_unlink_comm(c);
    if (c->base && c->base != MAP_FAILED) munmap(c->base, c->bytes);
    delete c;
}

}  // namespace lpcc
