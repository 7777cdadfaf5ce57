// Single-producer / multi-consumer message channel in POSIX shared memory: the
// control plane of the tensor-parallel serving engine (engine/tp_driver.py).
//
// Rank 0 owns the scheduler and publishes one message per runner call
// (prefill / decode rows / release ...); the TP follower ranks on the same
// node replay them. The reference's DeepSpeed-Inference / MII deployment
// (bloom-176b-deepspeed/files/isvc-patch.txt:85-92) synchronises its 8 ranks
// through torch.distributed; a pickled gloo broadcast per decode step puts a
// TCP round trip and rank skew on every token. Here a step costs the writer one
// memcpy + one release store, and a spinning follower sees it within
// microseconds -- no collective, no syscall on the hot path.
//
// Layout (one mapping, created by the writer, opened by readers):
//   Header   magic, geometry, writer pid (+ its pid namespace), head (next
//            sequence to write), closed flag, cursor[r] (next sequence reader r
//            will read), one cache line each
// A reader that times out checks that the writer process still exists: a
// writer killed without closing (OOM, SIGKILL) makes recv return -4, so the
// follower ranks exit instead of spinning forever on their GPUs.
//   Slot[n]  seq (published sequence + 1), length | LAST bit, payload
// A message larger than a slot is split into fragments (LAST on the final
// one). The writer reuses slot s for sequence q only after every reader's
// cursor passed q - nslots (back-pressure, bounded by `timeout_ms`).
// Ordering: payload stores, then a release store of slot.seq; readers acquire
// slot.seq before copying (x86-TSO or not, the atomics carry the ordering).
#include <errno.h>
#include <fcntl.h>
#include <signal.h>
#include <sched.h>
#include <stdint.h>
#include <string.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <time.h>
#include <unistd.h>

#include <atomic>
#include <new>

#if defined(__x86_64__)
#include <immintrin.h>
#define KCA_PAUSE() _mm_pause()
#else
#define KCA_PAUSE() ((void)0)
#endif

#define KCA_HOST_API extern "C" __attribute__((visibility("default")))

namespace {

constexpr uint64_t kMagic = 0x4b43414348414e31ull;  // "KCACHAN1"
constexpr int kMaxReaders = 64;
constexpr uint64_t kLast = 1ull << 63;

struct alignas(64) Line {
  std::atomic<uint64_t> v;
  char pad[64 - sizeof(std::atomic<uint64_t>)];
};

struct Header {
  uint64_t magic;
  uint64_t nslots;
  uint64_t slot_bytes;
  uint64_t readers;
  uint64_t writer_pid;
  uint64_t writer_pidns;  // inode of the writer's /proc/self/ns/pid (0: unknown)
  Line head;
  Line closed;
  Line cursor[kMaxReaders];
};

struct SlotHdr {
  std::atomic<uint64_t> seq;  // sequence + 1 once published
  uint64_t len;               // payload bytes | kLast
  char pad[48];
};

struct Chan {
  Header* h;
  size_t map_bytes;
  char* slots;
  int owner;
  char name[128];
};

inline SlotHdr* slot_at(Chan* c, uint64_t seq) {
  const uint64_t stride = sizeof(SlotHdr) + c->h->slot_bytes;
  return reinterpret_cast<SlotHdr*>(c->slots + (seq % c->h->nslots) * stride);
}

inline double now_ms() {
  timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return ts.tv_sec * 1e3 + ts.tv_nsec * 1e-6;
}

// spin, then yield, then sleep: a follower waiting between decode steps reacts
// within ~1 us while the step is in flight and backs off when the engine idles
struct Backoff {
  int n = 0;
  void wait() {
    if (n < 4000) {
      KCA_PAUSE();
    } else if (n < 8000) {
      sched_yield();
    } else {
      timespec ts{0, 50000};
      nanosleep(&ts, nullptr);
    }
    ++n;
  }
};

uint64_t pid_ns() {
  struct stat st;
  return stat("/proc/self/ns/pid", &st) == 0 ? (uint64_t)st.st_ino : 0;
}

// false only when the writer is provably gone: same pid namespace and no such process
bool writer_alive(const Header* h) {
  if (!h->writer_pid || !h->writer_pidns || h->writer_pidns != pid_ns()) return true;
  return !(kill((pid_t)h->writer_pid, 0) != 0 && errno == ESRCH);
}

size_t map_size(uint64_t nslots, uint64_t slot_bytes) {
  return sizeof(Header) + nslots * (sizeof(SlotHdr) + slot_bytes);
}

}  // namespace

// Writer: create (replacing a stale segment of the same name). Returns a handle or null.
KCA_HOST_API void* kca_chan_create(const char* name, long long nslots, long long slot_bytes, int readers) {
  if (!name || nslots < 2 || slot_bytes < 64 || slot_bytes % 64 || readers < 0 || readers > kMaxReaders ||
      strlen(name) >= 127)
    return nullptr;
  shm_unlink(name);
  const int fd = shm_open(name, O_CREAT | O_EXCL | O_RDWR, 0600);
  if (fd < 0) return nullptr;
  const size_t bytes = map_size((uint64_t)nslots, (uint64_t)slot_bytes);
  if (ftruncate(fd, (off_t)bytes) != 0) {
    close(fd);
    shm_unlink(name);
    return nullptr;
  }
  void* p = mmap(nullptr, bytes, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
  close(fd);
  if (p == MAP_FAILED) {
    shm_unlink(name);
    return nullptr;
  }
  memset(p, 0, sizeof(Header));
  Header* h = new (p) Header;
  h->nslots = (uint64_t)nslots;
  h->slot_bytes = (uint64_t)slot_bytes;
  h->readers = (uint64_t)readers;
  h->writer_pid = (uint64_t)getpid();
  h->writer_pidns = pid_ns();
  h->head.v.store(0, std::memory_order_relaxed);
  h->closed.v.store(0, std::memory_order_relaxed);
  for (int r = 0; r < kMaxReaders; ++r) h->cursor[r].v.store(0, std::memory_order_relaxed);
  char* slots = static_cast<char*>(p) + sizeof(Header);
  for (uint64_t s = 0; s < h->nslots; ++s) {
    SlotHdr* sh = new (slots + s * (sizeof(SlotHdr) + h->slot_bytes)) SlotHdr;
    sh->seq.store(0, std::memory_order_relaxed);
    sh->len = 0;
  }
  std::atomic_thread_fence(std::memory_order_seq_cst);
  __atomic_store_n(&h->magic, kMagic, __ATOMIC_RELEASE);  // readers check it last
  Chan* c = new Chan{h, bytes, slots, 1, {0}};
  strncpy(c->name, name, sizeof(c->name) - 1);
  return c;
}

// Reader: open an existing channel (waits up to timeout_ms for the writer to create it).
KCA_HOST_API void* kca_chan_open(const char* name, int timeout_ms) {
  if (!name || strlen(name) >= 127) return nullptr;
  const double t0 = now_ms();
  int fd = -1;
  for (;;) {
    fd = shm_open(name, O_RDWR, 0600);
    if (fd >= 0) {
      struct stat st;
      if (fstat(fd, &st) == 0 && (size_t)st.st_size >= sizeof(Header)) break;
      close(fd);
      fd = -1;
    }
    if (now_ms() - t0 > timeout_ms) return nullptr;
    timespec ts{0, 1000000};
    nanosleep(&ts, nullptr);
  }
  struct stat st;
  fstat(fd, &st);
  void* p = mmap(nullptr, (size_t)st.st_size, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
  close(fd);
  if (p == MAP_FAILED) return nullptr;
  Header* h = static_cast<Header*>(p);
  while (__atomic_load_n(&h->magic, __ATOMIC_ACQUIRE) != kMagic) {
    if (now_ms() - t0 > timeout_ms) {
      munmap(p, (size_t)st.st_size);
      return nullptr;
    }
    timespec ts{0, 1000000};
    nanosleep(&ts, nullptr);
  }
  if ((size_t)st.st_size < map_size(h->nslots, h->slot_bytes)) {
    munmap(p, (size_t)st.st_size);
    return nullptr;
  }
  Chan* c = new Chan{h, (size_t)st.st_size, static_cast<char*>(p) + sizeof(Header), 0, {0}};
  strncpy(c->name, name, sizeof(c->name) - 1);
  return c;
}

// 0 ok; -1 bad args; -2 timed out waiting for a sluggish reader; -3 closed.
KCA_HOST_API int kca_chan_send(void* hc, const void* data, long long len, int timeout_ms) {
  Chan* c = static_cast<Chan*>(hc);
  if (!c || !c->owner || len < 0 || (len > 0 && !data)) return -1;
  Header* h = c->h;
  const char* src = static_cast<const char*>(data);
  long long off = 0;
  const double t0 = now_ms();
  do {
    const uint64_t seq = h->head.v.load(std::memory_order_relaxed);
    // back-pressure: every reader must be past seq - nslots before the slot is reused
    if (seq >= h->nslots) {
      Backoff bo;
      for (;;) {
        uint64_t lo = UINT64_MAX;
        for (uint64_t r = 0; r < h->readers; ++r) {
          const uint64_t cur = h->cursor[r].v.load(std::memory_order_acquire);
          if (cur < lo) lo = cur;
        }
        if (h->readers == 0 || lo + h->nslots > seq) break;
        if (h->closed.v.load(std::memory_order_relaxed)) return -3;
        if (now_ms() - t0 > timeout_ms) return -2;
        bo.wait();
      }
    }
    SlotHdr* s = slot_at(c, seq);
    const long long n = (len - off) < (long long)h->slot_bytes ? (len - off) : (long long)h->slot_bytes;
    if (n > 0) memcpy(reinterpret_cast<char*>(s + 1), src + off, (size_t)n);
    off += n;
    s->len = (uint64_t)n | (off == len ? kLast : 0);
    s->seq.store(seq + 1, std::memory_order_release);
    h->head.v.store(seq + 1, std::memory_order_release);
  } while (off < len);
  return 0;
}

// Reader r: copy the next fragment into buf (cap >= the slot size) and set
// *last when it ends a message. Returns its length; -1 bad args; -2 timeout;
// -3 closed and drained; -4 the writer process died without closing. A fragment is consumed (its slot released to the
// writer) as soon as it is copied, so messages longer than the ring stream.
KCA_HOST_API long long kca_chan_recv(void* hc, int reader, void* buf, long long cap, int timeout_ms, int* last) {
  Chan* c = static_cast<Chan*>(hc);
  if (!c || reader < 0 || reader >= (int)c->h->readers || cap < (long long)c->h->slot_bytes || !last) return -1;
  Header* h = c->h;
  const uint64_t seq = h->cursor[reader].v.load(std::memory_order_relaxed);
  SlotHdr* s = slot_at(c, seq);
  const double t0 = now_ms();
  Backoff bo;
  while (s->seq.load(std::memory_order_acquire) != seq + 1) {
    if (h->closed.v.load(std::memory_order_acquire) && h->head.v.load(std::memory_order_acquire) <= seq) return -3;
    if (now_ms() - t0 > timeout_ms) return writer_alive(h) ? -2 : -4;
    bo.wait();
  }
  const uint64_t len = s->len;
  const long long n = (long long)(len & ~kLast);
  if (n > 0) memcpy(buf, reinterpret_cast<char*>(s + 1), (size_t)n);
  *last = (len & kLast) ? 1 : 0;
  h->cursor[reader].v.store(seq + 1, std::memory_order_release);
  return n;
}

KCA_HOST_API long long kca_chan_slot_bytes(void* hc) {
  Chan* c = static_cast<Chan*>(hc);
  return c ? (long long)c->h->slot_bytes : -1;
}

KCA_HOST_API void kca_chan_close(void* hc) {
  Chan* c = static_cast<Chan*>(hc);
  if (!c) return;
  if (c->owner) {
    c->h->closed.v.store(1, std::memory_order_release);
    shm_unlink(c->name);
  }
  munmap(c->h, c->map_bytes);
  delete c;
}
