// ishmem_amd — node-local shared-memory bootstrap (see bootstrap.h).
#include "bootstrap.h"

#include <errno.h>
#include <fcntl.h>
#include <signal.h>
#include <string.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <time.h>
#include <unistd.h>

#include <atomic>
#include <chrono>
#include <thread>

namespace ishmemi {

namespace {
constexpr uint64_t kMagic = 0x49534d454d414d44ull;  // "ISMEMAMD"

double now_ms()
{
    using namespace std::chrono;
    return duration<double, std::milli>(steady_clock::now().time_since_epoch()).count();
}

std::string sanitize(const std::string &key)
{
    std::string out = "/ishmem_amd_";
    for (char c : key) out += (isalnum((unsigned char) c) || c == '_' || c == '-') ? c : '_';
    return out.substr(0, 200);
}
}  // namespace

struct ShmBootstrap::Header {
    std::atomic<uint64_t> magic;
    int32_t npes;
    int32_t creator_pid;
    std::atomic<uint32_t> arrive;
    std::atomic<uint32_t> generation;
    char pad[64 - 24];
};
static_assert(sizeof(std::atomic<uint32_t>) == 4, "lock-free 32-bit atomics required");

char *ShmBootstrap::slot(int pe) const
{
    return static_cast<char *>(base_) + sizeof(Header) + (size_t) pe * kSlotBytes;
}

ShmBootstrap::~ShmBootstrap() { detach(); }

int ShmBootstrap::attach(int pe, int npes, const std::string &key, int timeout_ms, std::string &err)
{
    if (npes < 1 || pe < 0 || pe >= npes) {
        err = "bootstrap: invalid pe/npes";
        return 1;
    }
    pe_ = pe;
    npes_ = npes;
    timeout_ms_ = timeout_ms;
    name_ = sanitize(key);
    bytes_ = sizeof(Header) + (size_t) npes * kSlotBytes;
    const double t0 = now_ms();
    if (pe == 0) {
        int fd = shm_open(name_.c_str(), O_CREAT | O_EXCL | O_RDWR, 0600);
        if (fd < 0 && errno == EEXIST) {
            // A segment of this name exists: a crashed run's (its creator is gone: remove it) or
            // a live job's (refuse, instead of silently joining or unlinking another job).
            int32_t owner = 0;
            int efd = shm_open(name_.c_str(), O_RDONLY, 0600);
            if (efd >= 0) {
                struct stat st;
                if (fstat(efd, &st) == 0 && (size_t) st.st_size >= sizeof(Header)) {
                    void *b = mmap(nullptr, sizeof(Header), PROT_READ, MAP_SHARED, efd, 0);
                    if (b != MAP_FAILED) {
                        const Header *h = reinterpret_cast<const Header *>(b);
                        if (h->magic.load(std::memory_order_acquire) == kMagic) owner = h->creator_pid;
                        munmap(b, sizeof(Header));
                    }
                }
                close(efd);
            }
            if (owner > 0 && owner != (int32_t) getpid() && (kill(owner, 0) == 0 || errno == EPERM)) {
                err = "bootstrap: key '" + key + "' is in use by a live job (pid " +
                      std::to_string(owner) + "); set ISHMEM_BOOTSTRAP_KEY to a unique value";
                return 1;
            }
            shm_unlink(name_.c_str());
            fd = shm_open(name_.c_str(), O_CREAT | O_EXCL | O_RDWR, 0600);
        }
        if (fd < 0) {
            err = "bootstrap: shm_open(create) failed: " + std::string(strerror(errno));
            return 1;
        }
        if (ftruncate(fd, (off_t) bytes_) != 0) {
            err = "bootstrap: ftruncate failed";
            close(fd);
            return 1;
        }
        base_ = mmap(nullptr, bytes_, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
        close(fd);
        if (base_ == MAP_FAILED) {
            base_ = nullptr;
            err = "bootstrap: mmap failed";
            return 1;
        }
        Header *h = hdr();
        h->npes = npes;
        h->creator_pid = (int32_t) getpid();
        h->arrive.store(0, std::memory_order_relaxed);
        h->generation.store(0, std::memory_order_relaxed);
        h->magic.store(kMagic, std::memory_order_release);
    } else {
        for (;;) {
            if (now_ms() - t0 > timeout_ms) {
                err = "bootstrap: timed out waiting for PE 0 to create " + name_;
                return 1;
            }
            int fd = shm_open(name_.c_str(), O_RDWR, 0600);
            if (fd >= 0) {
                struct stat st;
                if (fstat(fd, &st) == 0 && (size_t) st.st_size >= bytes_) {
                    void *b = mmap(nullptr, bytes_, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
                    close(fd);
                    if (b != MAP_FAILED) {
                        Header *h = reinterpret_cast<Header *>(b);
                        const bool ready = h->magic.load(std::memory_order_acquire) == kMagic;
                        const bool alive =
                            ready && (kill(h->creator_pid, 0) == 0 || errno == EPERM);
                        if (ready && alive && h->npes == npes) {
                            base_ = b;
                            break;
                        }
                        munmap(b, bytes_);
                    }
                } else {
                    close(fd);
                }
            }
            std::this_thread::sleep_for(std::chrono::milliseconds(1));
        }
    }
    if (barrier(err) != 0) return 1;
    if (pe == 0) shm_unlink(name_.c_str());  // everyone is mapped; leave nothing behind
    return 0;
}

int ShmBootstrap::barrier(std::string &err)
{
    if (!base_) {
        err = "bootstrap: not attached";
        return 1;
    }
    Header *h = hdr();
    const uint32_t gen = h->generation.load(std::memory_order_acquire);
    if (h->arrive.fetch_add(1, std::memory_order_acq_rel) + 1 == (uint32_t) npes_) {
        h->arrive.store(0, std::memory_order_relaxed);
        h->generation.fetch_add(1, std::memory_order_acq_rel);
        return 0;
    }
    const double t0 = now_ms();
    unsigned spins = 0;
    while (h->generation.load(std::memory_order_acquire) == gen) {
        if (++spins > 1000) std::this_thread::sleep_for(std::chrono::microseconds(50));
        else std::this_thread::yield();
        if ((spins & 255) == 0 && now_ms() - t0 > timeout_ms_) {
            err = "bootstrap: barrier timed out";
            return 1;
        }
    }
    return 0;
}

int ShmBootstrap::allgather(const void *send, void *recv, size_t bytes, std::string &err)
{
    if (bytes > kSlotBytes) {
        err = "bootstrap: allgather payload too large";
        return 1;
    }
    memcpy(slot(pe_), send, bytes);
    if (barrier(err) != 0) return 1;
    for (int j = 0; j < npes_; ++j) memcpy(static_cast<char *>(recv) + (size_t) j * bytes, slot(j), bytes);
    return barrier(err);  // slots may be reused after everyone has read them
}

void ShmBootstrap::detach()
{
    if (base_) munmap(base_, bytes_);
    base_ = nullptr;
}

}  // namespace ishmemi
