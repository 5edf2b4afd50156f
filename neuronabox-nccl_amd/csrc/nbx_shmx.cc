// nbx_shmx.cc — see nbx_shmx.h.
#include "nbx_shmx.h"

#include <fcntl.h>
#include <immintrin.h>
#include <sched.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <atomic>
#include <chrono>
#include <cstring>

namespace nbx {
namespace {

constexpr uint64_t kMagic = 0x4e42585348585631ull;   // "NBXSHXV1"
constexpr size_t kLine = 64;

struct Header {
  std::atomic<uint64_t> magic;
  uint32_t n;
  uint32_t maxLen;
};

struct Slot {
  std::atomic<uint64_t> seq;
  uint64_t len;
  // payload follows
};

size_t roundUp(size_t x, size_t a) { return (x + a - 1) / a * a; }

}  // namespace

struct ShmExchange {
  void* base = nullptr;
  size_t bytes = 0;
  int rank = 0, n = 0;
  size_t maxLen = 0, slotStride = 0;
  uint64_t lastSeq = 0;   // this rank's previous exchange
  Header* hdr() const { return (Header*)base; }
  std::atomic<uint64_t>* ack(int j) const { return (std::atomic<uint64_t>*)((char*)base + kLine * (1 + j)); }
  Slot* slot(int j) const { return (Slot*)((char*)base + kLine * (1 + n) + slotStride * j); }
};

ShmExchange* shmxOpen(const char* name, int rank, int n, size_t maxLen, bool create) {
  auto* x = new ShmExchange();
  x->rank = rank;
  x->n = n;
  x->maxLen = maxLen;
  x->slotStride = roundUp(sizeof(Slot) + maxLen, kLine);
  x->bytes = kLine * (1 + n) + x->slotStride * n;
  int fd = create ? shm_open(name, O_CREAT | O_EXCL | O_RDWR, 0600) : shm_open(name, O_RDWR, 0600);
  if (fd < 0) {
    delete x;
    return nullptr;
  }
  if (create && ftruncate(fd, (off_t)x->bytes) != 0) {
    close(fd);
    shm_unlink(name);
    delete x;
    return nullptr;
  }
  struct stat st;
  if (fstat(fd, &st) != 0 || (size_t)st.st_size < x->bytes) {
    close(fd);
    delete x;
    return nullptr;
  }
  x->base = mmap(nullptr, x->bytes, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
  close(fd);
  if (x->base == MAP_FAILED) {
    if (create) shm_unlink(name);
    delete x;
    return nullptr;
  }
  if (create) {   // fresh segment is zero-filled: acks and seqs start at 0
    x->hdr()->n = (uint32_t)n;
    x->hdr()->maxLen = (uint32_t)maxLen;
    x->hdr()->magic.store(kMagic, std::memory_order_release);
  } else if (x->hdr()->magic.load(std::memory_order_acquire) != kMagic || x->hdr()->n != (uint32_t)n ||
             x->hdr()->maxLen != (uint32_t)maxLen) {
    shmxClose(x);
    return nullptr;
  }
  return x;
}

void shmxUnlink(const char* name) { shm_unlink(name); }

namespace {
// Spin until pred() (pause, then yield); false on timeout or abort.
template <class Pred>
bool spinUntil(Pred pred, double timeoutSec, const volatile int* abortWord) {
  if (pred()) return true;
  const auto t0 = std::chrono::steady_clock::now();
  for (uint32_t i = 1;; i++) {
    if (pred()) return true;
    if (i < 2048) {
      _mm_pause();
      continue;
    }
    sched_yield();
    if ((i & 255u) == 0u) {
      if (abortWord && *abortWord != 0) return false;
      if (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > timeoutSec) return false;
    }
  }
}
}  // namespace

ncclResult_t shmxAllGather(ShmExchange* x, uint64_t seq, const void* mine, size_t len, void* all, double timeoutSec,
                           const volatile int* abortWord) {
  if (len > x->maxLen || seq <= x->lastSeq) return ncclInternalError;
  const uint64_t prev = x->lastSeq;
  // nobody still reads this rank's previous payload
  for (int j = 0; j < x->n; j++)
    if (!spinUntil([&] { return x->ack(j)->load(std::memory_order_acquire) >= prev; }, timeoutSec, abortWord))
      return ncclRemoteError;
  Slot* s = x->slot(x->rank);
  s->len = len;
  std::memcpy((char*)s + sizeof(Slot), mine, len);
  s->seq.store(seq, std::memory_order_release);
  for (int j = 0; j < x->n; j++) {
    Slot* p = x->slot(j);
    if (!spinUntil([&] { return p->seq.load(std::memory_order_acquire) == seq; }, timeoutSec, abortWord))
      return ncclRemoteError;
    if (p->len != len) return ncclInvalidUsage;
    std::memcpy((char*)all + len * (size_t)j, (const char*)p + sizeof(Slot), len);
  }
  x->ack(x->rank)->store(seq, std::memory_order_release);
  x->lastSeq = seq;
  return ncclSuccess;
}

void shmxClose(ShmExchange* x) {
  if (!x) return;
  if (x->base && x->base != MAP_FAILED) munmap(x->base, x->bytes);
  delete x;
}

}  // namespace nbx
