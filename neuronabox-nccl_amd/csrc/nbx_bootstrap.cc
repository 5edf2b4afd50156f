// nbx_bootstrap.cc — see nbx_bootstrap.h.
//
// Wire format (all little-endian, one TCP stream per rank to the root):
//   hello   : {u64 key, i32 rank, i32 nranks}
//   round   : rank -> root {u64 len, len bytes};  root -> every rank {nranks x len bytes}
// The root relays rounds until any rank disconnects (comm destroy), then exits.
// Every blocking wait is bounded (NBX_BOOTSTRAP_TIMEOUT seconds, default 600).
#include "nbx_bootstrap.h"

#include <arpa/inet.h>
#include <errno.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <poll.h>
#include <sys/socket.h>
#include <unistd.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <thread>
#include <vector>

namespace nbx {
namespace {

constexpr char kMagic[8] = {'N', 'B', 'X', 'U', 'I', 'D', '0', '1'};

struct IdLayout {        // lives in ncclUniqueId::internal (128 bytes)
  char magic[8];
  uint64_t key;
  uint32_t addr;         // IPv4, network order; 0 = no root
  uint16_t port;         // network order
  uint16_t pad;
};
static_assert(sizeof(IdLayout) <= NCCL_UNIQUE_ID_BYTES, "id layout");

struct Hello {
  uint64_t key;
  int32_t rank;
  int32_t nranks;
};

thread_local const int* t_abort = nullptr;

bool aborted() { return t_abort && __atomic_load_n(t_abort, __ATOMIC_RELAXED) != 0; }

int timeoutMs() {
  const char* v = std::getenv("NBX_BOOTSTRAP_TIMEOUT");
  int s = (v && *v) ? std::atoi(v) : 600;
  return (s > 0 ? s : 600) * 1000;
}

// Read/write exactly n bytes, bounded by the timeout. Returns false on error/EOF/timeout.
bool ioAll(int fd, void* buf, size_t n, bool writing) {
  char* p = (char*)buf;
  const auto deadline = std::chrono::steady_clock::now() + std::chrono::milliseconds(timeoutMs());
  while (n > 0) {
    pollfd pf{fd, (short)(writing ? POLLOUT : POLLIN), 0};
    int left = (int)std::chrono::duration_cast<std::chrono::milliseconds>(deadline - std::chrono::steady_clock::now())
                   .count();
    if (left <= 0 || aborted()) return false;
    int pr = ::poll(&pf, 1, left < 100 ? left : 100);   // slices: an abort is seen within 0.1 s
    if (pr == 0) continue;
    if (pr < 0 && errno == EINTR) continue;
    if (pr <= 0) return false;
    ssize_t r = writing ? ::send(fd, p, n, MSG_NOSIGNAL) : ::recv(fd, p, n, 0);
    if (r < 0 && (errno == EINTR || errno == EAGAIN)) continue;
    if (r <= 0) return false;
    p += r;
    n -= (size_t)r;
  }
  return true;
}

void setNoDelay(int fd) {
  int one = 1;
  ::setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
}

void rootMain(int lfd, uint64_t key) {
  const int tmo = timeoutMs();
  std::vector<int> fds;
  int nranks = -1;
  // accept every rank (bounded: each wait for a connection times out)
  for (;;) {
    pollfd pf{lfd, POLLIN, 0};
    if (::poll(&pf, 1, tmo) <= 0) break;
    int cfd = ::accept(lfd, nullptr, nullptr);
    if (cfd < 0) continue;
    setNoDelay(cfd);
    Hello h;
    if (!ioAll(cfd, &h, sizeof(h), false) || h.key != key || h.nranks < 1 || h.rank < 0 || h.rank >= h.nranks ||
        (nranks >= 0 && h.nranks != nranks)) {
      ::close(cfd);
      continue;
    }
    if (nranks < 0) {
      nranks = h.nranks;
      fds.assign(nranks, -1);
    }
    if (fds[h.rank] != -1) {
      ::close(cfd);
      continue;
    }
    fds[h.rank] = cfd;
    int have = 0;
    for (int f : fds) have += f != -1;
    if (have == nranks) break;
  }
  ::close(lfd);
  bool ok = nranks > 0;
  for (int f : fds) ok &= f != -1;
  // relay rounds
  std::vector<char> all;
  while (ok) {
    uint64_t len = 0;
    for (int r = 0; r < nranks && ok; r++) {
      uint64_t l;
      if (!ioAll(fds[r], &l, sizeof(l), false)) {
        ok = false;
        break;
      }
      if (r == 0) {
        len = l;
        all.resize((size_t)len * (size_t)nranks);
      } else if (l != len) {
        ok = false;
        break;
      }
      if (len && !ioAll(fds[r], all.data() + (size_t)r * len, len, false)) ok = false;
    }
    for (int r = 0; r < nranks && ok; r++)
      if (!all.empty() && !ioAll(fds[r], all.data(), all.size(), true)) ok = false;
  }
  for (int f : fds)
    if (f != -1) ::close(f);
}

}  // namespace

struct Bootstrap {
  int fd = -1;
  int rank = 0;
  int nranks = 1;
};

bool bootstrapIdHasRoot(const ncclUniqueId& id) {
  IdLayout l;
  std::memcpy(&l, id.internal, sizeof(l));
  return std::memcmp(l.magic, kMagic, 8) == 0 && l.port != 0;
}

ncclResult_t bootstrapCreateRoot(ncclUniqueId* id) {
  std::memset(id, 0, sizeof(*id));
  IdLayout l{};
  std::memcpy(l.magic, kMagic, 8);
  std::random_device rd;
  l.key = ((uint64_t)rd() << 32) ^ rd();
  if (l.key == 0) l.key = 1;
  int lfd = ::socket(AF_INET, SOCK_STREAM, 0);
  if (lfd < 0) return ncclSystemError;
  int one = 1;
  ::setsockopt(lfd, SOL_SOCKET, SO_REUSEADDR, &one, sizeof(one));
  sockaddr_in sa{};
  sa.sin_family = AF_INET;
  const char* ip = std::getenv("NBX_BOOTSTRAP_ADDR");
  if (!ip || inet_pton(AF_INET, ip, &sa.sin_addr) != 1) sa.sin_addr.s_addr = htonl(INADDR_LOOPBACK);
  sa.sin_port = 0;
  socklen_t sl = sizeof(sa);
  if (::bind(lfd, (sockaddr*)&sa, sizeof(sa)) != 0 || ::listen(lfd, 256) != 0 ||
      ::getsockname(lfd, (sockaddr*)&sa, &sl) != 0) {
    ::close(lfd);
    return ncclSystemError;
  }
  l.addr = sa.sin_addr.s_addr;
  l.port = sa.sin_port;
  std::memcpy(id->internal, &l, sizeof(l));
  std::thread(rootMain, lfd, l.key).detach();
  return ncclSuccess;
}

ncclResult_t bootstrapConnect(const ncclUniqueId& id, int rank, int nranks, Bootstrap** out) {
  IdLayout l;
  std::memcpy(&l, id.internal, sizeof(l));
  if (std::memcmp(l.magic, kMagic, 8) != 0 || l.port == 0) return ncclInvalidArgument;
  sockaddr_in sa{};
  sa.sin_family = AF_INET;
  sa.sin_addr.s_addr = l.addr;
  sa.sin_port = l.port;
  const auto deadline = std::chrono::steady_clock::now() + std::chrono::milliseconds(timeoutMs());
  int fd = -1;
  for (;;) {
    fd = ::socket(AF_INET, SOCK_STREAM, 0);
    if (fd < 0) return ncclSystemError;
    if (::connect(fd, (sockaddr*)&sa, sizeof(sa)) == 0) break;
    ::close(fd);
    fd = -1;
    if (std::chrono::steady_clock::now() > deadline || aborted()) return ncclRemoteError;
    std::this_thread::sleep_for(std::chrono::milliseconds(20));
  }
  setNoDelay(fd);
  Hello h{l.key, rank, nranks};
  if (!ioAll(fd, &h, sizeof(h), true)) {
    ::close(fd);
    return ncclRemoteError;
  }
  Bootstrap* b = new Bootstrap();
  b->fd = fd;
  b->rank = rank;
  b->nranks = nranks;
  *out = b;
  return ncclSuccess;
}

ncclResult_t bootstrapAllGather(Bootstrap* b, const void* mine, size_t len, void* all) {
  uint64_t l = len;
  if (!ioAll(b->fd, &l, sizeof(l), true)) return ncclRemoteError;
  if (len && !ioAll(b->fd, const_cast<void*>(mine), len, true)) return ncclRemoteError;
  if (len && !ioAll(b->fd, all, len * (size_t)b->nranks, false)) return ncclRemoteError;
  return ncclSuccess;
}

void bootstrapSetAbortFlag(const int* flag) { t_abort = flag; }

void bootstrapClose(Bootstrap* b) {
  if (!b) return;
  if (b->fd >= 0) ::close(b->fd);
  delete b;
}

}  // namespace nbx
