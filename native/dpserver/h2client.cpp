// A gRPC unary client over HTTP/2 on a Unix socket (libnghttp2) — the simulator's kubelet.
//
// The kubelet's device manager calls Allocate through grpc-go, compiled; the simulated kubelet
// (sim/kubelet.py) used Python grpcio, whose client machinery added ~0.3 ms to every measured
// round trip. This client sends the call and reads the reply in C++, and stamps both ends
// itself (CLOCK_MONOTONIC), so the kubelet-side latency the bench reports is the plugin's plus
// the transport's, as the real kubelet sees it. One connection, one call at a time.
#include <ctype.h>
#include <errno.h>
#include <nghttp2/nghttp2.h>
#include <poll.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/socket.h>
#include <sys/un.h>
#include <time.h>
#include <unistd.h>

#include <mutex>
#include <string>

#include "dpserver.h"

namespace {

int64_t now_ns() {
  timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return (int64_t)ts.tv_sec * 1000000000 + ts.tv_nsec;
}

struct Call {
  int32_t sid = -1;
  std::string req, body, status, message, stamp;
  size_t off = 0;
  bool closed = false;
  uint32_t error = 0;
};

}  // namespace

struct gs_h2c {
  int fd = -1;
  nghttp2_session* sess = nullptr;
  std::mutex mu;
  Call* cur = nullptr;
  std::string wbuf;
};

namespace {

ssize_t req_read(nghttp2_session*, int32_t, uint8_t* buf, size_t len, uint32_t* flags, nghttp2_data_source*,
                 void* ud) {
  Call* c = static_cast<gs_h2c*>(ud)->cur;
  size_t n = std::min(len, c->req.size() - c->off);
  memcpy(buf, c->req.data() + c->off, n);
  c->off += n;
  if (c->off == c->req.size()) *flags |= NGHTTP2_DATA_FLAG_EOF;
  return (ssize_t)n;
}

std::string pct_decode(const std::string& v) {
  std::string o;
  for (size_t i = 0; i < v.size(); i++) {
    if (v[i] == '%' && i + 2 < v.size() && isxdigit((unsigned char)v[i + 1]) && isxdigit((unsigned char)v[i + 2])) {
      o += (char)strtol(v.substr(i + 1, 2).c_str(), nullptr, 16);
      i += 2;
    } else {
      o += v[i];
    }
  }
  return o;
}

int on_header(nghttp2_session*, const nghttp2_frame* f, const uint8_t* name, size_t nl, const uint8_t* value,
              size_t vl, uint8_t, void* ud) {
  Call* c = static_cast<gs_h2c*>(ud)->cur;
  if (!c || f->hd.stream_id != c->sid) return 0;
  std::string n((const char*)name, nl), v((const char*)value, vl);
  if (n == "grpc-status") c->status = v;
  else if (n == "grpc-message") c->message = pct_decode(v);
  else if (n == "gpushare-handler-ns") c->stamp = v;
  return 0;
}

int on_data(nghttp2_session*, uint8_t, int32_t sid, const uint8_t* d, size_t l, void* ud) {
  Call* c = static_cast<gs_h2c*>(ud)->cur;
  if (c && sid == c->sid) c->body.append((const char*)d, l);
  return 0;
}

int on_close(nghttp2_session*, int32_t sid, uint32_t err, void* ud) {
  Call* c = static_cast<gs_h2c*>(ud)->cur;
  if (c && sid == c->sid) {
    c->closed = true;
    c->error = err;
  }
  return 0;
}

bool flush(gs_h2c* h) {
  const uint8_t* data;
  ssize_t n;
  h->wbuf.clear();
  while ((n = nghttp2_session_mem_send(h->sess, &data)) > 0) h->wbuf.append((const char*)data, (size_t)n);
  if (n < 0) return false;
  size_t off = 0;
  while (off < h->wbuf.size()) {
    ssize_t w = send(h->fd, h->wbuf.data() + off, h->wbuf.size() - off, MSG_NOSIGNAL);
    if (w < 0) {
      if (errno == EINTR) continue;
      return false;
    }
    off += (size_t)w;
  }
  return true;
}

}  // namespace

extern "C" {

GS_DP_API gs_h2c* gs_h2c_connect(const char* socket_path) {
  sockaddr_un a{};
  if (strlen(socket_path) >= sizeof a.sun_path) return nullptr;
  int fd = socket(AF_UNIX, SOCK_STREAM | SOCK_CLOEXEC, 0);
  if (fd < 0) return nullptr;
  a.sun_family = AF_UNIX;
  strcpy(a.sun_path, socket_path);
  if (connect(fd, (sockaddr*)&a, sizeof a) != 0) {
    close(fd);
    return nullptr;
  }
  auto* h = new gs_h2c();
  h->fd = fd;
  nghttp2_session_callbacks* cb;
  nghttp2_session_callbacks_new(&cb);
  nghttp2_session_callbacks_set_on_header_callback(cb, on_header);
  nghttp2_session_callbacks_set_on_data_chunk_recv_callback(cb, on_data);
  nghttp2_session_callbacks_set_on_stream_close_callback(cb, on_close);
  nghttp2_session_client_new(&h->sess, cb, h);
  nghttp2_session_callbacks_del(cb);
  nghttp2_settings_entry iv[] = {{NGHTTP2_SETTINGS_INITIAL_WINDOW_SIZE, 1u << 20}};
  nghttp2_submit_settings(h->sess, NGHTTP2_FLAG_NONE, iv, 1);
  if (!flush(h)) {
    nghttp2_session_del(h->sess);
    close(fd);
    delete h;
    return nullptr;
  }
  return h;
}

// One unary call. Returns 0 (reply in out, grpc status in *status, handler stamp "in,out" in
// stamp) or -1 on a transport error / timeout. *t_send / *t_recv: CLOCK_MONOTONIC ns of the
// request's first byte written and of the reply complete.
GS_DP_API int gs_h2c_unary(gs_h2c* h, const char* path, const uint8_t* req, int len, uint8_t* out, int cap,
                           int* out_len, int* status, char* message, int mcap, char* stamp, int scap,
                           int timeout_ms, int64_t* t_send, int64_t* t_recv) {
  std::string framed(5, '\0');
  uint32_t l = (uint32_t)len;
  framed[1] = (char)(l >> 24), framed[2] = (char)(l >> 16), framed[3] = (char)(l >> 8), framed[4] = (char)l;
  framed.append((const char*)req, (size_t)len);
  return gs_h2c_call(h, path, (const uint8_t*)framed.data(), (int)framed.size(), out, cap, out_len, status,
                     message, mcap, stamp, scap, timeout_ms, t_send, t_recv);
}

// The same call with the request body sent as given (`body` is the whole DATA payload: gRPC
// length-prefixed messages, or anything else) — how the tests send what a broken or hostile
// client would.
GS_DP_API int gs_h2c_call(gs_h2c* h, const char* path, const uint8_t* body, int len, uint8_t* out, int cap,
                          int* out_len, int* status, char* message, int mcap, char* stamp, int scap,
                          int timeout_ms, int64_t* t_send, int64_t* t_recv) {
  std::lock_guard<std::mutex> lk(h->mu);
  Call c;
  c.req.assign((const char*)body, (size_t)len);
  h->cur = &c;
  std::string p = path;
  auto nv = [](const char* n, const std::string& v) {
    return nghttp2_nv{(uint8_t*)n, (uint8_t*)v.data(), strlen(n), v.size(), NGHTTP2_NV_FLAG_NONE};
  };
  std::string post = "POST", http = "http", auth = "localhost", ct = "application/grpc", te = "trailers",
              ua = "gpushare-sim-kubelet/1";
  nghttp2_nv hdr[] = {nv(":method", post), nv(":scheme", http), nv(":path", p), nv(":authority", auth),
                      nv("content-type", ct), nv("te", te), nv("user-agent", ua)};
  nghttp2_data_provider dp;
  dp.source.ptr = nullptr;
  dp.read_callback = req_read;
  c.sid = nghttp2_submit_request(h->sess, nullptr, hdr, 7, &dp, nullptr);
  if (c.sid < 0) return h->cur = nullptr, -1;
  *t_send = now_ns();
  if (!flush(h)) return h->cur = nullptr, -1;
  int64_t deadline = *t_send + (int64_t)timeout_ms * 1000000;
  uint8_t buf[65536];
  while (!c.closed) {
    int64_t left = (deadline - now_ns()) / 1000000;
    if (left < 0) return h->cur = nullptr, -1;
    pollfd pf{h->fd, POLLIN, 0};
    int r = poll(&pf, 1, (int)left + 1);
    if (r < 0 && errno == EINTR) continue;
    if (r <= 0) return h->cur = nullptr, -1;
    ssize_t n = recv(h->fd, buf, sizeof buf, 0);
    if (n <= 0) return h->cur = nullptr, -1;
    if (nghttp2_session_mem_recv(h->sess, buf, (size_t)n) < 0) return h->cur = nullptr, -1;
    if (!flush(h)) return h->cur = nullptr, -1;       // WINDOW_UPDATE / SETTINGS ACK / PING ACK
  }
  *t_recv = now_ns();
  h->cur = nullptr;
  if (c.error != 0 && c.status.empty()) return -1;
  *status = c.status.empty() ? 2 : atoi(c.status.c_str());
  snprintf(message, (size_t)mcap, "%s", c.message.c_str());
  snprintf(stamp, (size_t)scap, "%s", c.stamp.c_str());
  *out_len = 0;
  if (c.body.size() >= 5) {
    size_t m = c.body.size() - 5;
    if ((int)m > cap) return -1;
    memcpy(out, c.body.data() + 5, m);
    *out_len = (int)m;
  }
  return 0;
}

GS_DP_API void gs_h2c_close(gs_h2c* h) {
  if (!h) return;
  nghttp2_session_del(h->sess);
  close(h->fd);
  delete h;
}

}  // extern "C"
