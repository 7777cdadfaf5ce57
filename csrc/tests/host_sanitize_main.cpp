// ASan/UBSan harness for the host-side native runtime: the code
// that parses untrusted bytes -- the BPE pre-tokenizer/encoder (any UTF-8,
// valid or not), the context packer, the .tensors range reader, the HTTP
// response parser of the ranged-GET streamer (fed crafted, truncated and
// oversized responses by an in-process server) -- plus the host AdamW tails.
// Built and run by tools/build_ext.py --sanitize (tests/test_sanitize_cpu.py)
// with -fsanitize=address,undefined; any report aborts with a non-zero exit.
#include <arpa/inet.h>
#include <netinet/in.h>
#include <sys/socket.h>
#include <unistd.h>

#include <atomic>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <string>
#include <thread>
#include <vector>

extern "C" {
void* kca_bpe_new(const int32_t*, int, const int32_t*, const int32_t*, const int32_t*);
void kca_bpe_free(void*);
int64_t kca_bpe_encode(void*, const char*, int64_t, int32_t*, int64_t);
void* kca_packer_new(int, int, int, int, int, double);
void kca_packer_add(void*, const int32_t*, int64_t);
int kca_packer_write(void*, const char*, int64_t*);
void kca_packer_free(void*);
int kca_read_ranges(const char*, int, const int64_t*, const int64_t*, void**, int, int64_t, double*);
int kca_http_get_range(const char*, int, int, int, const char*, const char*, int64_t, int64_t, void*, int64_t*,
                       double);
int kca_http_stream(const char*, int, int, int, const char*, const char*, int, const int64_t*, const int64_t*,
                    void**, int, int, int64_t, double, double*);
int kca_host_adamw(float*, const float*, float*, float*, uint16_t*, const uint8_t*, int64_t, float, float, float,
                   float, float, float, float, float, int);
int kca_host_simd_level();
}

#define CHECK(c)                                                  \
  do {                                                            \
    if (!(c)) {                                                   \
      fprintf(stderr, "CHECK failed %s:%d: %s\n", __FILE__, __LINE__, #c); \
      std::exit(3);                                               \
    }                                                             \
  } while (0)

static std::mt19937_64 rng(1234);

static void test_bpe() {
  // vocab: 256 byte symbols, then merges (a,b)->id for random pairs
  int32_t byte_ids[256];
  for (int i = 0; i < 256; ++i) byte_ids[i] = (i == 0xC0 || i == 0xFF) ? -1 : i;
  std::vector<int32_t> L, R, M;
  for (int r = 0; r < 400; ++r) {
    L.push_back((int32_t)(rng() % 300));
    R.push_back((int32_t)(rng() % 300));
    M.push_back(256 + r);
  }
  void* h = kca_bpe_new(byte_ids, (int)L.size(), L.data(), R.data(), M.data());
  std::vector<int32_t> out(1 << 16);
  const char* alphabet[] = {"a", "Z", "9", " ", "\n", "\t", "'", "'s", "é", "日", "👍", "\xC0", "\xFF", "\xE2\x82",
                            "\xF0\x9F", "\x80", "  ", "ll", "\xE3\x80\x80"};
  for (int it = 0; it < 20000; ++it) {
    std::string s;
    const int n = (int)(rng() % 40);
    for (int k = 0; k < n; ++k) s += alphabet[rng() % (sizeof(alphabet) / sizeof(*alphabet))];
    if (rng() % 4 == 0 && !s.empty()) s.resize(rng() % s.size());  // cut mid-sequence
    const int64_t need = kca_bpe_encode(h, s.data(), (int64_t)s.size(), nullptr, 0);
    CHECK(need >= 0 && need <= (int64_t)s.size());
    const int64_t cap = need > 0 ? (int64_t)(rng() % (need + 1)) : 0;  // short output buffers too
    const int64_t got = kca_bpe_encode(h, s.data(), (int64_t)s.size(), out.data(), cap);
    CHECK(got == need);
  }
  kca_bpe_free(h);
}

static void test_packer() {
  char path[] = "/tmp/kca_san_pack_XXXXXX";
  int fd = mkstemp(path);
  CHECK(fd >= 0);
  close(fd);
  for (int it = 0; it < 200; ++it) {
    const int ctx = 1 + (int)(rng() % 64);
    void* p = kca_packer_new(ctx, (int)(rng() % 5), (int)(rng() % 80) - 10, 0, 1, 25.0 + (double)(rng() % 100));
    for (int d = 0; d < 20; ++d) {
      std::vector<int32_t> t(rng() % 200);
      for (auto& x : t) x = (int32_t)(rng() % 6);
      kca_packer_add(p, t.data(), (int64_t)t.size());
    }
    int64_t st[2];
    CHECK(kca_packer_write(p, path, st) == 0);
    CHECK(st[1] <= st[0]);
    kca_packer_free(p);
  }
  unlink(path);
}

static void test_read_ranges() {
  char path[] = "/tmp/kca_san_rr_XXXXXX";
  int fd = mkstemp(path);
  CHECK(fd >= 0);
  std::vector<uint8_t> data(1 << 20);
  for (auto& b : data) b = (uint8_t)rng();
  CHECK(write(fd, data.data(), data.size()) == (ssize_t)data.size());
  close(fd);
  for (int it = 0; it < 50; ++it) {
    const int n = 1 + (int)(rng() % 16);
    std::vector<int64_t> offs(n), lens(n);
    std::vector<std::vector<uint8_t>> bufs(n);
    std::vector<void*> dsts(n);
    for (int i = 0; i < n; ++i) {
      offs[i] = (int64_t)(rng() % data.size());
      lens[i] = (int64_t)(rng() % (data.size() - offs[i] + 1));
      bufs[i].resize(lens[i] + 1);
      dsts[i] = bufs[i].data();
    }
    double st[2];
    CHECK(kca_read_ranges(path, n, offs.data(), lens.data(), dsts.data(), 1 + (int)(rng() % 6),
                          1 + (int64_t)(rng() % 100000), st) == 0);
    for (int i = 0; i < n; ++i) CHECK(memcmp(bufs[i].data(), data.data() + offs[i], lens[i]) == 0);
  }
  // past EOF must fail cleanly
  int64_t o = (int64_t)data.size() - 10, l = 100;
  std::vector<uint8_t> b(100);
  void* d = b.data();
  CHECK(kca_read_ranges(path, 1, &o, &l, &d, 1, 0, nullptr) != 0);
  CHECK(kca_read_ranges("/nonexistent/kca", 1, &o, &l, &d, 1, 0, nullptr) != 0);
  unlink(path);
}

// ---- HTTP: a one-connection-at-a-time server that answers from a script
static std::vector<uint8_t> g_obj;
static std::atomic<int> g_mode{0};

static void serve(int lfd) {
  for (;;) {
    int c = accept(lfd, nullptr, nullptr);
    if (c < 0) return;
    for (;;) {
      std::string req;
      char buf[4096];
      while (req.find("\r\n\r\n") == std::string::npos) {
        ssize_t r = recv(c, buf, sizeof buf, 0);
        if (r <= 0) break;
        req.append(buf, (size_t)r);
      }
      if (req.find("\r\n\r\n") == std::string::npos) break;
      long long a = 0, z = 0;
      const char* rg = strstr(req.c_str(), "Range: bytes=");
      if (rg) sscanf(rg, "Range: bytes=%lld-%lld", &a, &z);
      if (z >= (long long)g_obj.size()) z = (long long)g_obj.size() - 1;
      const int mode = g_mode.load();
      std::string head;
      const long long n = z - a + 1;
      if (mode == 0) {  // well-formed 206
        head = "HTTP/1.1 206 Partial Content\r\nContent-Length: " + std::to_string(n) + "\r\nContent-Range: bytes " +
               std::to_string(a) + "-" + std::to_string(z) + "/" + std::to_string(g_obj.size()) + "\r\n\r\n";
        send(c, head.data(), head.size(), MSG_NOSIGNAL);
        send(c, g_obj.data() + a, (size_t)n, MSG_NOSIGNAL);
        continue;
      }
      if (mode == 1) head = "HTTP/1.1 206 OK\r\nContent-Length: " + std::to_string(n + 7) + "\r\n\r\n";  // wrong length
      if (mode == 2) head = "HTTP/1.1 206 OK\r\n\r\n";                                                  // no length
      if (mode == 3) head = "HTTP/1.1 404 Not Found\r\nContent-Length: 0\r\n\r\n";
      if (mode == 4) head = "garbage without status line\r\n\r\n";
      if (mode == 5) head = std::string(100000, 'X');                                                     // header flood
      if (mode == 6) head = "HTTP/1.1 206 OK\r\nContent-Length: " + std::to_string(n) + "\r\n\r\n";     // short body
      send(c, head.data(), head.size(), MSG_NOSIGNAL);
      if (mode == 6) send(c, g_obj.data() + a, (size_t)(n / 2), MSG_NOSIGNAL);
      break;
    }
    close(c);
  }
}

static void test_http() {
  g_obj.resize(300000);
  for (auto& b : g_obj) b = (uint8_t)rng();
  int lfd = socket(AF_INET, SOCK_STREAM, 0);
  sockaddr_in addr{};
  addr.sin_family = AF_INET;
  addr.sin_addr.s_addr = htonl(INADDR_LOOPBACK);
  CHECK(bind(lfd, (sockaddr*)&addr, sizeof addr) == 0);
  socklen_t al = sizeof addr;
  getsockname(lfd, (sockaddr*)&addr, &al);
  listen(lfd, 16);
  const int port = ntohs(addr.sin_port);
  std::thread th(serve, lfd);
  // good path: several ranges over keep-alive connections into host memory
  std::vector<uint8_t> out(g_obj.size());
  int64_t offs[3] = {0, 1000, 200000}, lens[3] = {1000, 199000, 100000};
  void* dsts[3] = {out.data(), out.data() + 1000, out.data() + 200000};
  double st[2];
  CHECK(kca_http_stream("127.0.0.1", port, 0, 0, "/obj", "", 3, offs, lens, dsts, -1, 1, 7777, 5.0, st) == 0);
  CHECK(memcmp(out.data(), g_obj.data(), g_obj.size()) == 0);
  int64_t total = 0;
  CHECK(kca_http_get_range("127.0.0.1", port, 0, 0, "/obj", "X-A: b\r\n", 5, 10, out.data(), &total, 5.0) == 0);
  CHECK(total == (int64_t)g_obj.size() && memcmp(out.data(), g_obj.data() + 5, 10) == 0);
  // malformed responses: must return an error, never touch memory out of bounds
  for (int mode = 1; mode <= 6; ++mode) {
    g_mode = mode;
    std::vector<uint8_t> small(64);
    const int rc = kca_http_get_range("127.0.0.1", port, 0, 0, "/obj", "", 0, 64, small.data(), nullptr, 2.0);
    CHECK(rc != 0);
  }
  CHECK(kca_http_get_range("127.0.0.1", 1, 0, 0, "/", "", 0, 1, out.data(), nullptr, 1.0) != 0);  // refused
  shutdown(lfd, SHUT_RDWR);
  close(lfd);
  th.join();
}

static void test_adamw() {
  for (int it = 0; it < 40; ++it) {
    const int64_t n = 1 + (int64_t)(rng() % 5000);
    std::vector<float> p(n), g(n), m(n), v(n);
    std::vector<uint16_t> pb(n);
    std::vector<uint8_t> mask((n + 63) / 64, 1);
    for (int64_t i = 0; i < n; ++i) {
      p[i] = (float)(rng() % 1000) / 1000.f;
      g[i] = (float)((int)(rng() % 2001) - 1000) / 1000.f;
    }
    for (int lvl : {1, 256, 512}) {
      if (lvl > 1 && lvl > kca_host_simd_level()) continue;
      CHECK(kca_host_adamw(p.data(), g.data(), m.data(), v.data(), pb.data(), (it & 1) ? mask.data() : nullptr, n,
                           1e-3f, 0.9f, 0.999f, 1e-8f, 0.01f, 0.1f, 0.001f, 1.f, lvl) == 0);
    }
    for (int64_t i = 0; i < n; ++i) CHECK(std::isfinite(p[i]));
  }
}

int main() {
  test_bpe();
  test_packer();
  test_read_ranges();
  test_http();
  test_adamw();
  printf("host sanitize harness: OK\n");
  return 0;
}
