// Fast weight streamer: storage -> pinned host ring -> HBM (K25 / N17).
//
// Replaces tensorizer's TensorDeserializer(plaid_mode=True) that the
// reference uses for cold starts (online-inference/tensorizer-isvc/
// tensorizer_hf_isvc/load_model.py:56-59; stable-diffusion/service/
// service.py:87-93). Design for MI355X (288 GB HBM per GPU, PCIe Gen5 x16):
//
//   * the load is a flat list of (file_offset, nbytes, device_ptr) copies --
//     the caller preallocates every parameter in HBM, so no allocator work or
//     module construction sits on the critical path;
//   * copies are split into chunks (default 64 MiB) handed to N reader
//     threads; each thread owns its pinned buffers (hipHostMalloc) and a HIP
//     stream, preads a chunk (O_DIRECT when 4 KiB aligned, bypassing the page
//     cache, else buffered), then hipMemcpyAsync's it while the next pread
//     runs -- double buffering per thread keeps the PCIe link and the storage
//     read both busy;
//   * stats (bytes, seconds) are returned for the GB/s line the reference
//     prints (load_model.py:63-73).
//
// C ABI, loaded with ctypes after torch (same HIP runtime soname).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fcntl.h>
#include <mutex>
#include <thread>
#include <unistd.h>
#include <vector>

#define KCA_HOST_API extern "C" __attribute__((visibility("default")))

namespace {

struct Chunk {
  int64_t off;
  int64_t len;
  char* dst;  // device or host pointer
};

constexpr int64_t kAlign = 4096;

bool pread_full(int fd, char* buf, int64_t len, int64_t off) {
  int64_t done = 0;
  while (done < len) {
    ssize_t r = ::pread(fd, buf + done, (size_t)(len - done), (off_t)(off + done));
    if (r < 0) {
      if (errno == EINTR) continue;
      return false;
    }
    if (r == 0) return false;
    done += r;
  }
  return true;
}

std::vector<Chunk> make_chunks(int n, const int64_t* offs, const int64_t* lens, void** dsts,
                               int64_t chunk) {
  std::vector<Chunk> v;
  for (int i = 0; i < n; ++i) {
    for (int64_t p = 0; p < lens[i]; p += chunk) {
      int64_t l = std::min(chunk, lens[i] - p);
      v.push_back({offs[i] + p, l, (char*)dsts[i] + p});
    }
  }
  // issue in file order: sequential storage reads
  std::sort(v.begin(), v.end(), [](const Chunk& a, const Chunk& b) { return a.off < b.off; });
  return v;
}

double now_s() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

}  // namespace

// Parallel read of byte ranges straight into host memory (CPU loads, tests).
KCA_HOST_API int kca_read_ranges(const char* path, int n, const int64_t* offs, const int64_t* lens,
                                 void** dsts, int n_threads, int64_t chunk, double* stats) {
  int fd = ::open(path, O_RDONLY);
  if (fd < 0) return 1;
  if (chunk <= 0) chunk = 64 << 20;
  auto chunks = make_chunks(n, offs, lens, dsts, chunk);
  std::atomic<size_t> next{0};
  std::atomic<int> err{0};
  double t0 = now_s();
  auto work = [&]() {
    for (;;) {
      size_t i = next.fetch_add(1);
      if (i >= chunks.size() || err.load()) return;
      if (!pread_full(fd, chunks[i].dst, chunks[i].len, chunks[i].off)) err = 2;
    }
  };
  n_threads = std::max(1, std::min(n_threads, 64));
  std::vector<std::thread> th;
  for (int t = 0; t < n_threads; ++t) th.emplace_back(work);
  for (auto& t : th) t.join();
  ::close(fd);
  if (stats) {
    int64_t tot = 0;
    for (int i = 0; i < n; ++i) tot += lens[i];
    stats[0] = (double)tot;
    stats[1] = now_s() - t0;
  }
  return err.load();
}

// Stream byte ranges of `path` into device memory on `device`.
// stats[0] = bytes, stats[1] = seconds (wall, including the final sync), stats[2] = payload bytes
// read with O_DIRECT, stats[3] = payload bytes that took the buffered path (O_DIRECT not requested,
// refused at open, or a short read) -- the record says which path a "cold" number measured.
KCA_HOST_API int kca_stream_to_device(const char* path, int n, const int64_t* offs,
                                      const int64_t* lens, void** dev_dsts, int device,
                                      int n_threads, int64_t chunk, int use_odirect,
                                      double* stats) {
  if (chunk <= 0) chunk = 64 << 20;
  chunk = (chunk + kAlign - 1) / kAlign * kAlign;
  int fd_buf = ::open(path, O_RDONLY);
  if (fd_buf < 0) return 1;
  int fd_dir = use_odirect ? ::open(path, O_RDONLY | O_DIRECT) : -1;
  auto chunks = make_chunks(n, offs, lens, dev_dsts, chunk);
  n_threads = std::max(1, std::min(n_threads, 32));
  std::atomic<size_t> next{0};
  std::atomic<int> err{0};
  std::atomic<int64_t> direct_bytes{0}, buffered_bytes{0};
  double t0 = now_s();
  auto work = [&]() {
    if (hipSetDevice(device) != hipSuccess) { err = 3; return; }
    hipStream_t st;
    if (hipStreamCreateWithFlags(&st, hipStreamNonBlocking) != hipSuccess) { err = 3; return; }
    // two pinned buffers (+ alignment slack) and their completion events
    char* buf[2] = {nullptr, nullptr};
    hipEvent_t ev[2];
    for (int b = 0; b < 2; ++b) {
      if (hipHostMalloc((void**)&buf[b], chunk + 2 * kAlign, hipHostMallocDefault) != hipSuccess) {
        err = 4;
        return;
      }
      hipEventCreateWithFlags(&ev[b], hipEventDisableTiming);
      hipEventRecord(ev[b], st);
    }
    int cur = 0;
    for (;;) {
      size_t i = next.fetch_add(1);
      if (i >= chunks.size() || err.load()) break;
      const Chunk& c = chunks[i];
      hipEventSynchronize(ev[cur]);  // buffer free again (its previous copy finished)
      char* hb = buf[cur];
      int64_t lead = 0;
      bool ok;
      if (fd_dir >= 0) {
        // aligned superset read; the payload starts `lead` bytes in
        int64_t a0 = c.off / kAlign * kAlign;
        lead = c.off - a0;
        int64_t alen = (lead + c.len + kAlign - 1) / kAlign * kAlign;
        ssize_t r = ::pread(fd_dir, hb, (size_t)alen, (off_t)a0);
        ok = r >= lead + c.len;
        if (ok) {
          direct_bytes += c.len;
        } else {  // short read at EOF or O_DIRECT refusal: buffered fallback
          lead = 0;
          ok = pread_full(fd_buf, hb, c.len, c.off);
          buffered_bytes += c.len;
        }
      } else {
        ok = pread_full(fd_buf, hb, c.len, c.off);
        buffered_bytes += c.len;
      }
      if (!ok) { err = 2; break; }
      if (hipMemcpyAsync(c.dst, hb + lead, (size_t)c.len, hipMemcpyHostToDevice, st) != hipSuccess) {
        err = 5;
        break;
      }
      hipEventRecord(ev[cur], st);
      cur ^= 1;
    }
    hipStreamSynchronize(st);
    for (int b = 0; b < 2; ++b) {
      hipEventDestroy(ev[b]);
      hipHostFree(buf[b]);
    }
    hipStreamDestroy(st);
  };
  std::vector<std::thread> th;
  for (int t = 0; t < n_threads; ++t) th.emplace_back(work);
  for (auto& t : th) t.join();
  ::close(fd_buf);
  if (fd_dir >= 0) ::close(fd_dir);
  if (stats) {
    int64_t tot = 0;
    for (int i = 0; i < n; ++i) tot += lens[i];
    stats[0] = (double)tot;
    stats[1] = now_s() - t0;
    stats[2] = (double)direct_bytes.load();
    stats[3] = (double)buffered_bytes.load();
  }
  return err.load();
}

// Raw storage read rate of `path` (BASELINE.md weight load: "saturate the storage read rate"): the
// whole file read with O_DIRECT (page cache bypassed) by n_threads into per-thread aligned host
// buffers, nothing copied to the device -- the ceiling kca_stream_to_device's pipeline can reach.
// stats[0] = bytes, stats[1] = seconds.
KCA_HOST_API int kca_read_bandwidth(const char* path, int n_threads, int64_t chunk, int use_odirect,
                                    double* stats) {
  if (chunk <= 0) chunk = 64 << 20;
  chunk = (chunk + kAlign - 1) / kAlign * kAlign;
  int fd = ::open(path, O_RDONLY | (use_odirect ? O_DIRECT : 0));
  if (fd < 0) return 1;
  const off_t size = ::lseek(fd, 0, SEEK_END);
  if (size <= 0) {
    ::close(fd);
    return 1;
  }
  n_threads = std::max(1, std::min(n_threads, 64));
  const int64_t n_chunks = (size + chunk - 1) / chunk;
  std::atomic<int64_t> next{0};
  std::atomic<int> err{0};
  double t0 = now_s();
  auto work = [&]() {
    void* buf = nullptr;
    if (posix_memalign(&buf, kAlign, (size_t)chunk) != 0) {
      err = 4;
      return;
    }
    for (;;) {
      const int64_t i = next.fetch_add(1);
      if (i >= n_chunks || err.load()) break;
      const int64_t off = i * chunk, len = std::min<int64_t>(chunk, size - off);
      const int64_t alen = (len + kAlign - 1) / kAlign * kAlign;  // O_DIRECT: whole blocks (EOF short)
      int64_t done = 0;
      while (done < len) {
        const ssize_t r = ::pread(fd, (char*)buf + done, (size_t)(alen - done), (off_t)(off + done));
        if (r < 0 && errno == EINTR) continue;
        if (r <= 0) break;
        done += r;
      }
      if (done < len) err = 2;
    }
    free(buf);
  };
  std::vector<std::thread> th;
  for (int t = 0; t < n_threads; ++t) th.emplace_back(work);
  for (auto& t : th) t.join();
  ::close(fd);
  if (stats) {
    stats[0] = (double)size;
    stats[1] = now_s() - t0;
  }
  return err.load();
}
