// HTTP(S) / S3 ranged-GET weight streamer: object store -> pinned host ring -> HBM
// (N17 / K25: tensorizer's CURLStreamFile + TensorDeserializer, used by the
// reference to stream weights straight from S3 -- finetuner-workflow/finetuner/
// finetuner.py:395-410,802-815; stable-diffusion/service/service.py:87-93;
// tensorizer-isvc/tensorizer_hf_isvc/load_model.py:56-59).
//
// Same plan as the file streamer (tensor_stream.cpp): the caller preallocates
// every tensor and passes a flat list of (object offset, nbytes, destination)
// ranges; the ranges are cut into chunks that N worker threads claim from a
// shared queue. Each worker keeps ONE persistent HTTP/1.1 keep-alive
// connection (TLS via OpenSSL when https), sends `Range: bytes=a-b` GETs and
// receives each body straight into one of its two pinned buffers, then
// hipMemcpyAsync's it to HBM while the next range downloads. N connections in
// parallel is what saturates an object store (one TCP stream tops out far
// below a 100 Gb NIC). S3 is plain HTTPS path-style addressing; SigV4
// headers, when credentials are configured, are computed by the caller
// (io/remote.py) and passed through `extra_headers`.
//
// No libcurl headers exist in the image, so this is a small self-contained
// client: blocking sockets with SO_RCVTIMEO, Content-Length bodies only (range
// responses are never chunked), one redirect-free endpoint, retry of a failed
// range on a fresh connection.
#include <hip/hip_runtime.h>
#include <netdb.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <openssl/err.h>
#include <openssl/ssl.h>
#include <openssl/x509v3.h>
#include <poll.h>
#include <sys/socket.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <cerrno>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fcntl.h>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#define KCA_HOST_API extern "C" __attribute__((visibility("default")))

namespace {

double now_s() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

struct Endpoint {
  std::string host;
  int port;
  bool tls;
  bool verify;
  std::string path;
  std::string headers;  // extra request headers, each terminated by \r\n
  double timeout_s;
};

SSL_CTX* ssl_ctx(bool verify) {
  static std::once_flag once;
  static SSL_CTX* ctx[2] = {nullptr, nullptr};
  std::call_once(once, [] {
    for (int v = 0; v < 2; ++v) {
      SSL_CTX* c = SSL_CTX_new(TLS_client_method());
      if (!c) continue;
      SSL_CTX_set_min_proto_version(c, TLS1_2_VERSION);
      if (v) {
        SSL_CTX_set_default_verify_paths(c);
        SSL_CTX_set_verify(c, SSL_VERIFY_PEER, nullptr);
      } else {
        SSL_CTX_set_verify(c, SSL_VERIFY_NONE, nullptr);
      }
      ctx[v] = c;
    }
  });
  return ctx[verify ? 1 : 0];
}

class Conn {
 public:
  explicit Conn(const Endpoint& ep) : ep_(ep) {}
  ~Conn() { close_(); }

  // GET [off, off+len) into dst. Returns 0, or an error code (HTTP status if >= 100).
  int get_range(int64_t off, int64_t len, char* dst, int64_t* total_size = nullptr) {
    for (int attempt = 0; attempt < 3; ++attempt) {
      if (fd_ < 0 && !connect_()) continue;
      int rc = request_(off, len, dst, total_size);
      if (rc == 0) return 0;
      close_();
      if (rc >= 400 && rc != 408 && rc != 429 && rc < 500) return rc;  // client errors are final
      last_ = rc;
    }
    return last_ ? last_ : 1;
  }

 private:
  bool connect_() {
    char port[16];
    snprintf(port, sizeof port, "%d", ep_.port);
    addrinfo hints{}, *res = nullptr;
    hints.ai_family = AF_UNSPEC;
    hints.ai_socktype = SOCK_STREAM;
    if (getaddrinfo(ep_.host.c_str(), port, &hints, &res) != 0) { last_ = 2; return false; }
    int fd = -1;
    for (addrinfo* a = res; a; a = a->ai_next) {
      fd = ::socket(a->ai_family, a->ai_socktype, a->ai_protocol);
      if (fd < 0) continue;
      // bounded connect: non-blocking + poll, then back to blocking with I/O timeouts
      int fl = fcntl(fd, F_GETFL, 0);
      fcntl(fd, F_SETFL, fl | O_NONBLOCK);
      int r = ::connect(fd, a->ai_addr, a->ai_addrlen);
      if (r < 0 && errno == EINPROGRESS) {
        pollfd p{fd, POLLOUT, 0};
        r = poll(&p, 1, (int)(ep_.timeout_s * 1000)) == 1 ? 0 : -1;
        int soerr = 0;
        socklen_t sl = sizeof soerr;
        if (r == 0 && (getsockopt(fd, SOL_SOCKET, SO_ERROR, &soerr, &sl) != 0 || soerr != 0)) r = -1;
      }
      if (r == 0) {
        fcntl(fd, F_SETFL, fl);
        break;
      }
      ::close(fd);
      fd = -1;
    }
    freeaddrinfo(res);
    if (fd < 0) { last_ = 3; return false; }
    int one = 1, rcv = 16 << 20;
    setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof one);
    setsockopt(fd, SOL_SOCKET, SO_RCVBUF, &rcv, sizeof rcv);
    timeval tv{(time_t)ep_.timeout_s, (suseconds_t)((ep_.timeout_s - (int64_t)ep_.timeout_s) * 1e6)};
    setsockopt(fd, SOL_SOCKET, SO_RCVTIMEO, &tv, sizeof tv);
    setsockopt(fd, SOL_SOCKET, SO_SNDTIMEO, &tv, sizeof tv);
    fd_ = fd;
    if (ep_.tls) {
      SSL_CTX* c = ssl_ctx(ep_.verify);
      if (!c) { close_(); last_ = 4; return false; }
      ssl_ = SSL_new(c);
      SSL_set_fd(ssl_, fd_);
      SSL_set_tlsext_host_name(ssl_, ep_.host.c_str());
      if (ep_.verify) X509_VERIFY_PARAM_set1_host(SSL_get0_param(ssl_), ep_.host.c_str(), 0);
      if (SSL_connect(ssl_) != 1) { close_(); last_ = 5; return false; }
    }
    buf_.clear();
    return true;
  }

  void close_() {
    if (ssl_) {
      SSL_free(ssl_);
      ssl_ = nullptr;
    }
    if (fd_ >= 0) ::close(fd_);
    fd_ = -1;
    buf_.clear();
  }

  ssize_t send_(const char* p, size_t n) {
    if (ssl_) return SSL_write(ssl_, p, (int)n);
    return ::send(fd_, p, n, MSG_NOSIGNAL);
  }
  ssize_t recv_(char* p, size_t n) {
    if (ssl_) return SSL_read(ssl_, p, (int)std::min<size_t>(n, 1 << 30));
    for (;;) {
      ssize_t r = ::recv(fd_, p, n, 0);
      if (r < 0 && errno == EINTR) continue;
      return r;
    }
  }

  int request_(int64_t off, int64_t len, char* dst, int64_t* total_size) {
    char range[96];
    snprintf(range, sizeof range, "Range: bytes=%lld-%lld\r\n", (long long)off, (long long)(off + len - 1));
    std::string req = "GET " + ep_.path + " HTTP/1.1\r\nHost: " + ep_.host + "\r\n" + range +
                      "Connection: keep-alive\r\nAccept-Encoding: identity\r\nUser-Agent: kca-stream/1\r\n" +
                      ep_.headers + "\r\n";
    size_t sent = 0;
    while (sent < req.size()) {
      ssize_t r = send_(req.data() + sent, req.size() - sent);
      if (r <= 0) return 10;
      sent += (size_t)r;
    }
    // headers (keep any body bytes that arrived with them in buf_)
    size_t hend;
    for (;;) {
      hend = buf_.find("\r\n\r\n");
      if (hend != std::string::npos) break;
      if (buf_.size() > (1 << 16)) return 11;
      char tmp[8192];
      ssize_t r = recv_(tmp, sizeof tmp);
      if (r <= 0) return 12;
      buf_.append(tmp, (size_t)r);
    }
    std::string head = buf_.substr(0, hend);
    buf_.erase(0, hend + 4);
    int status = 0;
    if (sscanf(head.c_str(), "HTTP/%*d.%*d %d", &status) != 1) return 13;
    std::string lower = head;
    std::transform(lower.begin(), lower.end(), lower.begin(), ::tolower);
    auto header = [&](const char* key) -> std::string {
      size_t p = lower.find(std::string("\r\n") + key + ":");
      if (p == std::string::npos) return "";
      p += 3 + strlen(key);
      size_t e = lower.find("\r\n", p);
      std::string v = head.substr(p, e == std::string::npos ? std::string::npos : e - p);
      size_t a = v.find_first_not_of(" \t");
      return a == std::string::npos ? "" : v.substr(a);
    };
    std::string cl = header("content-length");
    if (cl.empty()) return 14;
    const int64_t body = std::atoll(cl.c_str());
    const bool keep = lower.find("\r\nconnection: close") == std::string::npos;
    if (status != 206 && !(status == 200 && off == 0 && body == len)) {
      // error status: the body is not read; the caller closes this connection
      // (its state is unknown past the headers) and reports the status
      return status >= 100 ? status : 15;
    }
    if (body != len) return 16;
    if (total_size) {
      std::string cr = header("content-range");  // bytes a-b/total
      size_t sl = cr.find('/');
      *total_size = (sl != std::string::npos) ? std::atoll(cr.c_str() + sl + 1) : body;
    }
    int64_t got = std::min<int64_t>((int64_t)buf_.size(), len);
    memcpy(dst, buf_.data(), (size_t)got);
    buf_.erase(0, (size_t)got);
    while (got < len) {
      ssize_t r = recv_(dst + got, (size_t)(len - got));
      if (r <= 0) return 17;
      got += r;
    }
    if (!keep) close_();
    return 0;
  }

  Endpoint ep_;
  int fd_ = -1;
  SSL* ssl_ = nullptr;
  std::string buf_;
  int last_ = 0;
};

Endpoint make_ep(const char* host, int port, int tls, int verify, const char* path, const char* headers,
                 double timeout_s) {
  return Endpoint{host, port, tls != 0, verify != 0, path, headers ? headers : "", timeout_s > 0 ? timeout_s : 30.0};
}

struct Chunk {
  int64_t off, len;
  char* dst;
};

}  // namespace

// One ranged GET into host memory (header reads, existence probes).
// Returns 0, a transport error code (< 100) or the HTTP status (>= 100).
// total_size (optional) receives the object size from Content-Range.
KCA_HOST_API int kca_http_get_range(const char* host, int port, int tls, int verify, const char* path,
                                    const char* headers, int64_t off, int64_t len, void* dst, int64_t* total_size,
                                    double timeout_s) {
  Endpoint ep = make_ep(host, port, tls, verify, path, headers, timeout_s);
  Conn c(ep);
  return c.get_range(off, len, (char*)dst, total_size);
}

// Stream byte ranges of an HTTP object into device memory (device >= 0) or
// host memory (device < 0) over n_threads keep-alive connections.
// stats[0] = bytes, stats[1] = seconds.
KCA_HOST_API int kca_http_stream(const char* host, int port, int tls, int verify, const char* path,
                                 const char* headers, int n, const int64_t* offs, const int64_t* lens, void** dsts,
                                 int device, int n_threads, int64_t chunk, double timeout_s, double* stats) {
  if (chunk <= 0) chunk = 16 << 20;
  Endpoint ep = make_ep(host, port, tls, verify, path, headers, timeout_s);
  std::vector<Chunk> chunks;
  for (int i = 0; i < n; ++i)
    for (int64_t p = 0; p < lens[i]; p += chunk)
      chunks.push_back({offs[i] + p, std::min(chunk, lens[i] - p), (char*)dsts[i] + p});
  std::sort(chunks.begin(), chunks.end(), [](const Chunk& a, const Chunk& b) { return a.off < b.off; });
  n_threads = std::max(1, std::min(n_threads, 64));
  std::atomic<size_t> next{0};
  std::atomic<int> err{0};
  const double t0 = now_s();
  auto work = [&]() {
    Conn conn(ep);
    if (device < 0) {  // host destination: receive in place
      for (;;) {
        size_t i = next.fetch_add(1);
        if (i >= chunks.size() || err.load()) return;
        int rc = conn.get_range(chunks[i].off, chunks[i].len, chunks[i].dst);
        if (rc) { err = rc; return; }
      }
    }
    if (hipSetDevice(device) != hipSuccess) { err = 90; return; }
    hipStream_t st;
    if (hipStreamCreateWithFlags(&st, hipStreamNonBlocking) != hipSuccess) { err = 90; return; }
    char* buf[2] = {nullptr, nullptr};
    hipEvent_t ev[2];
    for (int b = 0; b < 2; ++b) {
      if (hipHostMalloc((void**)&buf[b], (size_t)chunk, hipHostMallocDefault) != hipSuccess) { err = 91; return; }
      hipEventCreateWithFlags(&ev[b], hipEventDisableTiming);
      hipEventRecord(ev[b], st);
    }
    int cur = 0;
    for (;;) {
      size_t i = next.fetch_add(1);
      if (i >= chunks.size() || err.load()) break;
      const Chunk& c = chunks[i];
      hipEventSynchronize(ev[cur]);  // this pinned buffer's previous upload finished
      int rc = conn.get_range(c.off, c.len, buf[cur]);
      if (rc) { err = rc; break; }
      if (hipMemcpyAsync(c.dst, buf[cur], (size_t)c.len, hipMemcpyHostToDevice, st) != hipSuccess) {
        err = 92;
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
  if (stats) {
    int64_t tot = 0;
    for (int i = 0; i < n; ++i) tot += lens[i];
    stats[0] = (double)tot;
    stats[1] = now_s() - t0;
  }
  return err.load();
}
