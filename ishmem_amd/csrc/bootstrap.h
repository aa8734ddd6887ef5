// ishmem_amd — node-local bootstrap: handle exchange + host barrier over POSIX shared memory.
//
// Replaces, for this path, the reference's host runtime (MPI / OpenSHMEM / PMI behind
// src/runtime.h:22-84) whose only role on the reduce path's setup is exchanging the heap IPC
// handles (src/ipc.cpp:123-233, pidfd / Unix-socket fd passing) and host barriers during init.
// Everything here is one node (the north star is one 8 x MI355X node), so a shared-memory
// segment is sufficient and needs no MPI.
#pragma once
#include <stddef.h>

#include <string>

namespace ishmemi {

class ShmBootstrap {
  public:
    static constexpr size_t kSlotBytes = 4096;

    ShmBootstrap() = default;
    ~ShmBootstrap();
    ShmBootstrap(const ShmBootstrap &) = delete;
    ShmBootstrap &operator=(const ShmBootstrap &) = delete;

    // Attach as `pe` of `npes`.  PE 0 creates the segment; the others wait for it (up to
    // timeout_ms).  Returns 0 or nonzero with `err` filled.
    int attach(int pe, int npes, const std::string &key, int timeout_ms, std::string &err);
    // Every PE contributes `bytes` (<= kSlotBytes); `recv` receives npes * bytes in PE order.
    int allgather(const void *send, void *recv, size_t bytes, std::string &err);
    int barrier(std::string &err);
    void detach();
    bool attached() const { return base_ != nullptr; }

  private:
    struct Header;
    Header *hdr() const { return reinterpret_cast<Header *>(base_); }
    char *slot(int pe) const;

    void *base_ = nullptr;
    size_t bytes_ = 0;
    int pe_ = -1, npes_ = 0;
    int timeout_ms_ = 60000;
    std::string name_;
};

}  // namespace ishmemi
