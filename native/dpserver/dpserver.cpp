// libgpushare_dpserver.so — native DevicePlugin gRPC server (see dpserver.h).
//
// Reference: the plugin's gRPC server is grpc-go (pkg/gpu/nvidia/server.go:114-142), Allocate
// runs under one global lock with a LIST + PATCH inside (allocate.go:60-152). The MI355X build
// answers the common Allocate here: the Python engine keeps, for every candidate pod, its
// answer already serialized (alloc/engine.py "prepared answers"), and this library serves the
// pick without entering the interpreter — the grpcio server's per-call cost (a poller thread,
// an executor thread and the GIL twice) was most of the kubelet-side latency (bench.py
// allocate_breakdown_p50_ms).
//
// Layout
//   * an accept thread, and one thread per kubelet connection running an nghttp2 server
//     session over the socket (HTTP/2 framing, HPACK, flow control); a connection's eventfd
//     wakes its thread for replies from Python and device-list changes;
//   * unary requests complete in on_frame_recv: Allocate tries the fast table, everything
//     else is queued for the Python handler threads (gs_dp_next) and answered from their
//     gs_dp_reply; ListAndWatch streams the device list Python sets;
//   * the fast table (published by Python) answers an Allocate exactly when the engine's own
//     fast path would: one container, table built at the current pod-cache version and engine
//     generation, no possible replay of its fake IDs, and the first unclaimed candidate of the
//     request's size is a single-container pod (with admission identity on, also the only
//     one). The pick is claimed, its journal record written, the reply sent, and the claim
//     reported to the engine (gs_dp_taken_next) for the write-behind PATCH and bookkeeping.
#include "dpserver.h"

#include <errno.h>
#include <fcntl.h>
#include <nghttp2/nghttp2.h>
#include <poll.h>
#include <sched.h>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/eventfd.h>
#include <sys/mman.h>
#include <sys/socket.h>
#include <sys/stat.h>
#include <sys/un.h>
#include <time.h>
#include <unistd.h>

#include <atomic>
#include <chrono>
#include <condition_variable>
#include <deque>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <unordered_map>
#include <unordered_set>
#include <vector>

namespace {

int64_t mono_ns() {
  timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return (int64_t)ts.tv_sec * 1000000000 + ts.tv_nsec;
}

// Condition-variable deadlines on the system clock: libstdc++ waits on steady-clock deadlines
// with pthread_cond_clockwait, which ThreadSanitizer builds of this toolchain do not intercept
// (the mutex hand-over inside the wait goes unseen and every queue access reads as a race).
// The waits are short timeouts, so a wall-clock step only shortens or lengthens one of them.
std::chrono::system_clock::time_point deadline_us(long long us) {
  return std::chrono::system_clock::now() + std::chrono::microseconds(us);
}

double wall_s() {
  timespec ts;
  clock_gettime(CLOCK_REALTIME, &ts);
  return (double)ts.tv_sec + ts.tv_nsec / 1e9;
}

const char* kB64 = "ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789+/";

// ---- protobuf: AllocateRequest { repeated ContainerAllocateRequest container_requests = 1 }
//                ContainerAllocateRequest { repeated string devices_ids = 1 } -----------------
bool varint(const uint8_t*& p, const uint8_t* e, uint64_t* v) {
  uint64_t r = 0;
  for (int s = 0; s < 64 && p < e; s += 7) {
    uint8_t b = *p++;
    r |= (uint64_t)(b & 0x7f) << s;
    if (!(b & 0x80)) {
      *v = r;
      return true;
    }
  }
  return false;
}

bool skip_field(const uint8_t*& p, const uint8_t* e, int wt) {
  uint64_t v;
  switch (wt) {
    case 0: return varint(p, e, &v);
    case 1: if (e - p < 8) return false; p += 8; return true;
    case 2: if (!varint(p, e, &v) || (uint64_t)(e - p) < v) return false; p += v; return true;
    case 5: if (e - p < 4) return false; p += 4; return true;
    default: return false;
  }
}

// Per container, its device IDs (views into the buffer). False on a malformed message.
bool parse_allocate(const uint8_t* p, const uint8_t* e, std::vector<std::vector<std::string>>* out) {
  while (p < e) {
    uint64_t tag;
    if (!varint(p, e, &tag)) return false;
    int field = (int)(tag >> 3), wt = (int)(tag & 7);
    if (field == 1 && wt == 2) {
      uint64_t len;
      if (!varint(p, e, &len) || (uint64_t)(e - p) < len) return false;
      const uint8_t* q = p;
      const uint8_t* qe = p + len;
      p = qe;
      out->emplace_back();
      while (q < qe) {
        uint64_t t2;
        if (!varint(q, qe, &t2)) return false;
        if ((t2 >> 3) == 1 && (t2 & 7) == 2) {
          uint64_t l2;
          if (!varint(q, qe, &l2) || (uint64_t)(qe - q) < l2) return false;
          out->back().emplace_back((const char*)q, (size_t)l2);
          q += l2;
        } else if (!skip_field(q, qe, (int)(t2 & 7))) {
          return false;
        }
      }
    } else if (!skip_field(p, e, wt)) {
      return false;
    }
  }
  return true;
}

// ---- the fast table ---------------------------------------------------------------------
// blob: u64 version, u64 gen, u32 flags (bit 0: admission identity on — an answer needs the
// only unclaimed candidate of its size; bit 31: no table, every Allocate to the engine), u32 entries, u32 replay ids, then per entry
// {u32 size, u8 multi, u32 len + uid, u32 len + response bytes, u32 len + journal head}, then
// per replay id {u32 len + id} (fake IDs of journaled answers whose pod may still be retried).
struct Entry {
  uint32_t size = 0;
  bool multi = false;
  bool taken = false;
  std::string uid, body, head;
};

struct Table {
  bool valid = false;
  uint64_t version = 0, gen = 0;
  uint32_t flags = 0;
  std::vector<Entry> entries;
  std::unordered_set<std::string> replay;
};

struct Reader {
  const uint8_t* p;
  const uint8_t* e;
  bool ok = true;
  uint32_t u32() {
    if (e - p < 4) return ok = false, 0;
    uint32_t v;
    memcpy(&v, p, 4);
    p += 4;
    return v;
  }
  uint64_t u64() {
    if (e - p < 8) return ok = false, 0;
    uint64_t v;
    memcpy(&v, p, 8);
    p += 8;
    return v;
  }
  uint8_t u8() {
    if (e - p < 1) return ok = false, 0;
    return *p++;
  }
  std::string str() {
    uint32_t n = u32();
    if (!ok || (uint32_t)(e - p) < n) return ok = false, std::string();
    std::string s((const char*)p, n);
    p += n;
    return s;
  }
};

bool parse_table(const uint8_t* blob, int len, Table* t) {
  Reader r{blob, blob + len};
  t->version = r.u64();
  t->gen = r.u64();
  t->flags = r.u32();
  uint32_t n = r.u32(), nr = r.u32();
  if (!r.ok || n > (1u << 20) || nr > (1u << 24)) return false;
  t->entries.resize(n);
  for (auto& en : t->entries) {
    en.size = r.u32();
    en.multi = r.u8() != 0;
    en.uid = r.str();
    en.body = r.str();
    en.head = r.str();
  }
  t->replay.reserve(nr);
  for (uint32_t i = 0; i < nr; ++i) t->replay.insert(r.str());
  return r.ok && r.p == r.e;
}

// ---- server state -----------------------------------------------------------------------
struct Conn;

struct Reply {
  int32_t stream;
  int status;
  std::string message, body;
};

struct Fwd {
  int64_t id;
  std::weak_ptr<Conn> conn;
  int32_t stream;
  std::string method, body;
  int64_t t_in;
  int64_t deadline = 0;     // CLOCK_MONOTONIC ns from the client's grpc-timeout; 0 = none
};

struct Taken {
  std::string uid, req;
  double t;
  uint64_t handler_ns;
  int64_t t_in;            // CLOCK_MONOTONIC ns the request was complete
  uint64_t watch_wait_ns;  // waited for a table holding a pod of this size
  uint64_t table_wait_ns;  // waited for the table to catch up with the pod cache
};

struct Counters {
  std::atomic<uint64_t> fast{0}, forwarded{0}, forwarded_allocate{0}, stale{0}, blocked{0}, replay{0}, nomatch{0}, multi{0},
      ambiguous{0}, shape{0}, journal{0}, waited{0}, law_sends{0}, conns{0}, unknown{0}, older{0}, watch_waits{0}, wait_ns{0}, expired{0},
      lock_ns{0}, journal_ns{0}, answer_ns{0};
};

}  // namespace

struct gs_dp {
  std::string path;
  int lfd = -1;
  std::atomic<bool> stopping{false};
  std::thread acceptor;
  std::mutex conns_mu;
  std::vector<std::shared_ptr<Conn>> conns;   // live ones; ended ones are joined and dropped at the next accept

  // requests for Python
  std::mutex q_mu;
  std::condition_variable q_cv;
  std::deque<std::shared_ptr<Fwd>> queue;
  std::unordered_map<int64_t, std::shared_ptr<Fwd>> inflight;
  int64_t next_id = 1;

  // ListAndWatch
  std::mutex dev_mu;
  std::string devices;   // the gRPC-framed message (5-byte prefix + ListAndWatchResponse)
  uint64_t dev_gen = 0;

  // fast path (mu guards the table, the versions, the block count and the journal)
  std::mutex mu;
  std::condition_variable cv;
  Table table;
  uint64_t cur_version = 0, cur_gen = 0;
  int blocked = 0;
  int fast_wait_us = 300;
  int watch_wait_us = 2000;
  // until then (CLOCK_MONOTONIC ns) connection threads busy-poll instead of sleeping: set when
  // a pod the kubelet is about to admit was published (gs_dp_spin). A core that slept pays
  // tens of microseconds of wake-up and cold caches on the Allocate path (measured: building
  // one journal record takes 1 us hot, 30 us on a core idle for 300 ms)
  std::atomic<int64_t> spin_until{0};
  // bumped (under mu) by everything a table wait depends on: a spinning waiter watches it
  // without the lock, so it never contends with the publisher it is waiting for
  std::atomic<uint64_t> table_seq{0};
  uint64_t pub_seq = 0;                  // tables published (under mu)   // an Allocate with no candidate yet waits this long for the pod watch
  // fake IDs of native answers -> when: a kubelet retry of them is for the engine (replay),
  // kept until a published replay set covers them (or for 30 s, by when the engine has)
  std::unordered_map<std::string, int64_t> answered_ids;
  std::unordered_set<std::string> taken_uids;     // claimed (natively or by the engine)
  std::deque<Taken> taken;
  std::condition_variable taken_cv;
  // journal
  int jfd = -1;
  uint8_t* jmap = nullptr;
  uint64_t jsize = 0, joff = 0;

  Counters n;
};

namespace {

struct Stream {
  std::string path, body, out;
  size_t off = 0;
  bool law = false;         // ListAndWatch: stays open, more messages follow
  bool unary_done = false;  // the unary response is fully queued
  int status = 0;
  std::string message;
  int64_t t_in = 0, t_out = 0;
  bool stamp = false;
  bool too_big = false;     // the request passed kMaxRequest: its bytes are dropped, answered RESOURCE_EXHAUSTED
  int64_t deadline = 0;     // grpc-timeout, as CLOCK_MONOTONIC ns
};

// gRPC "grpc-timeout": up to 8 digits and a unit (H, M, S, m, u, n). 0 when absent or malformed.
int64_t parse_grpc_timeout_ns(const uint8_t* v, size_t n) {
  if (n < 2 || n > 9) return 0;
  int64_t x = 0;
  for (size_t i = 0; i + 1 < n; ++i) {
    if (v[i] < '0' || v[i] > '9') return 0;
    x = x * 10 + (v[i] - '0');
  }
  int64_t unit;
  switch (v[n - 1]) {
    case 'H': unit = 3600 * 1000000000LL; break;
    case 'M': unit = 60 * 1000000000LL; break;
    case 'S': unit = 1000000000LL; break;
    case 'm': unit = 1000000LL; break;
    case 'u': unit = 1000LL; break;
    case 'n': unit = 1; break;
    default: return 0;
  }
  int64_t ns;
  if (__builtin_mul_overflow(x, unit, &ns) || ns > (int64_t)1 << 61) return 0;   // years: no deadline
  return ns;
}

// Larger requests are refused (gRPC's default receive limit is 4 MiB; Python's handler buffer is 8)
constexpr size_t kMaxRequest = (8u << 20) + 5;

struct Conn {
  gs_dp* srv;
  int fd;
  int efd = -1;                      // wakes the thread; open while any reference (a reply in flight) lives
  std::thread th;                    // serve_conn; joined by the acceptor once done, or at stop
  std::weak_ptr<Conn> self;
  std::atomic<bool> done{false};     // the connection ended (its thread exits)
  bool wake_taken = false;           // a native answer went out this turn (conn thread only)
  nghttp2_session* sess = nullptr;
  std::map<int32_t, Stream> streams;
  std::mutex out_mu;                 // replies from Python threads
  std::vector<Reply> outbox;
  uint64_t sent_dev_gen = 0;
  std::atomic<bool> closing{false};
  ~Conn() {
    if (efd >= 0) close(efd);
  }
};

void wake(Conn* c) {
  uint64_t one = 1;
  ssize_t r = write(c->efd, &one, sizeof one);
  (void)r;
}

std::string grpc_frame(const std::string& msg) {
  std::string f(5, '\0');
  uint32_t l = (uint32_t)msg.size();
  f[1] = (char)(l >> 24);
  f[2] = (char)(l >> 16);
  f[3] = (char)(l >> 8);
  f[4] = (char)l;
  return f + msg;
}

nghttp2_nv nv(const char* n, const std::string& v) {
  return nghttp2_nv{(uint8_t*)n, (uint8_t*)v.data(), strlen(n), v.size(), NGHTTP2_NV_FLAG_NONE};
}

const std::string kStatus200 = "200", kCtype = "application/grpc";

ssize_t read_cb(nghttp2_session* sess, int32_t sid, uint8_t* buf, size_t len, uint32_t* flags,
                nghttp2_data_source*, void* ud) {
  Conn* c = static_cast<Conn*>(ud);
  auto it = c->streams.find(sid);
  if (it == c->streams.end()) {
    *flags |= NGHTTP2_DATA_FLAG_EOF;
    return 0;
  }
  Stream& st = it->second;
  size_t n = std::min(len, st.out.size() - st.off);
  memcpy(buf, st.out.data() + st.off, n);
  st.off += n;
  if (st.off == st.out.size()) {
    if (st.law && !c->closing.load()) {
      st.out.clear();
      st.off = 0;
      if (n == 0) return NGHTTP2_ERR_DEFERRED;
      return (ssize_t)n;
    }
    *flags |= NGHTTP2_DATA_FLAG_EOF | NGHTTP2_DATA_FLAG_NO_END_STREAM;
    std::string code = std::to_string(st.status);
    std::vector<nghttp2_nv> tr{nv("grpc-status", code)};
    if (!st.message.empty()) tr.push_back(nv("grpc-message", st.message));
    std::string stamp;
    if (st.stamp) {
      // handler entry / exit (CLOCK_MONOTONIC ns), the same trailer the Python server sends
      stamp = std::to_string(st.t_in) + "," + std::to_string(st.t_out);
      tr.push_back(nv("gpushare-handler-ns", stamp));
    }
    nghttp2_submit_trailer(sess, sid, tr.data(), tr.size());
  }
  return (ssize_t)n;
}

// A unary answer: headers, one message, trailers (status 0); or trailers-only on an error.
// grpc-message is percent-encoded (gRPC over HTTP/2 spec): an exception text with a newline
// would otherwise be an invalid header value that grpc-go rejects, losing the status
std::string pct_encode(const std::string& m) {
  static const char* hex = "0123456789ABCDEF";
  std::string o;
  for (unsigned char ch : m) {
    if (ch >= 0x20 && ch <= 0x7e && ch != '%') {
      o += (char)ch;
    } else {
      o += '%';
      o += hex[ch >> 4];
      o += hex[ch & 15];
    }
  }
  return o;
}

void respond(Conn* c, int32_t sid, int status, const std::string& message, const std::string& body, bool stamp) {
  auto it = c->streams.find(sid);
  if (it == c->streams.end()) return;  // the client went away
  Stream& st = it->second;
  st.t_out = mono_ns();
  st.stamp = stamp;
  if (status != 0) {
    std::string code = std::to_string(status), msg = pct_encode(message);
    std::vector<nghttp2_nv> h{nv(":status", kStatus200), nv("content-type", kCtype), nv("grpc-status", code)};
    if (!msg.empty()) h.push_back(nv("grpc-message", msg));
    nghttp2_submit_response(c->sess, sid, h.data(), h.size(), nullptr);
    return;
  }
  st.out = grpc_frame(body);
  st.off = 0;
  st.status = 0;
  st.unary_done = true;
  nghttp2_nv h[] = {nv(":status", kStatus200), nv("content-type", kCtype)};
  nghttp2_data_provider dp;
  dp.source.ptr = nullptr;
  dp.read_callback = read_cb;
  nghttp2_submit_response(c->sess, sid, h, 2, &dp);
}

// ---- the Allocate fast path ---------------------------------------------------------------
// The record is written straight into the mapping (no intermediate string): the entry's
// prepared head, the wall time, the request in base64. The terminating newline goes last, so
// a record cut short by a crash is never a complete line.
bool journal_append(gs_dp* s, const Entry& en, const std::string& req, double t) {
  if (!s->jmap) return true;
  char tb[48];
  int tl = snprintf(tb, sizeof tb, "%.6f", t);
  static const char kReq[] = ",\"req\":\"";
  size_t b64 = (req.size() + 2) / 3 * 4;
  size_t need = en.head.size() + (size_t)tl + sizeof kReq - 1 + b64 + 3;
  if (s->joff + need >= s->jsize) return false;  // full: the engine rotates it
  uint8_t* p = s->jmap + s->joff;
  memcpy(p, en.head.data(), en.head.size()), p += en.head.size();
  memcpy(p, tb, (size_t)tl), p += tl;
  memcpy(p, kReq, sizeof kReq - 1), p += sizeof kReq - 1;
  const uint8_t* r = (const uint8_t*)req.data();
  size_t n = req.size(), i = 0;
  for (; i + 3 <= n; i += 3) {
    uint32_t v = (uint32_t)r[i] << 16 | (uint32_t)r[i + 1] << 8 | r[i + 2];
    p[0] = kB64[v >> 18], p[1] = kB64[v >> 12 & 63], p[2] = kB64[v >> 6 & 63], p[3] = kB64[v & 63];
    p += 4;
  }
  if (n - i == 1) {
    uint32_t v = (uint32_t)r[i] << 16;
    p[0] = kB64[v >> 18], p[1] = kB64[v >> 12 & 63], p[2] = '=', p[3] = '=';
    p += 4;
  } else if (n - i == 2) {
    uint32_t v = (uint32_t)r[i] << 16 | (uint32_t)r[i + 1] << 8;
    p[0] = kB64[v >> 18], p[1] = kB64[v >> 12 & 63], p[2] = kB64[v >> 6 & 63], p[3] = '=';
    p += 4;
  }
  p[0] = '"', p[1] = '}';
  __atomic_thread_fence(__ATOMIC_RELEASE);
  p[2] = '\n';
  s->joff += need;
  return true;
}

enum Decline { kOk = 0, kReplay, kMulti, kAmbiguous, kNoMatch };

// Caller holds s->mu. The entry to answer (kOk), or why the engine must decide.
Decline pick(gs_dp* s, const std::vector<std::string>& ids, const Entry** out) {
  Table& t = s->table;
  size_t n = ids.size();
  for (const auto& id : ids)
    if (t.replay.count(id) || s->answered_ids.count(id)) return kReplay;
  Entry* first = nullptr;
  for (auto& en : t.entries) {
    if (en.size != n || en.taken || s->taken_uids.count(en.uid)) continue;
    if (!first) {
      first = &en;
      if (en.multi) return kMulti;                  // a multi-container pod first in line
      if (!(t.flags & 1)) break;
    } else {
      return kAmbiguous;                            // which one is for admission identity to say
    }
  }
  if (!first) return kNoMatch;
  *out = first;
  return kOk;
}

void count_decline(gs_dp* s, Decline d) {
  switch (d) {
    case kReplay: s->n.replay++; break;
    case kMulti: s->n.multi++; break;
    case kAmbiguous: s->n.ambiguous++; break;
    case kNoMatch: s->n.nomatch++; break;
    default: break;
  }
}

// Wait (s->mu held via lk) until pred() or `us` passed: spinning while the busy-poll window is
// open (a sleeping thread wakes up cold), on the condition variable otherwise.
template <class Pred>
void wait_for_table(gs_dp* s, std::unique_lock<std::mutex>& lk, int us, Pred pred) {
  if (s->spin_until.load(std::memory_order_relaxed) > mono_ns()) {
    int64_t dl = mono_ns() + (int64_t)us * 1000;
    while (!pred() && mono_ns() < dl) {
      uint64_t seq = s->table_seq.load(std::memory_order_acquire);
      lk.unlock();
      while (s->table_seq.load(std::memory_order_acquire) == seq && mono_ns() < dl && !s->stopping.load())
        sched_yield();
      lk.lock();
    }
    return;
  }
  s->cv.wait_until(lk, deadline_us(us), pred);
}

bool table_current(gs_dp* s) {
  return s->table.valid && s->blocked == 0 && s->table.version == s->cur_version && s->table.gen == s->cur_gen;
}

// Answer an Allocate from the table if the engine would answer it the same way. True = done.
bool fast_allocate(Conn* c, int32_t sid, const std::string& body, int64_t t_in) {
  gs_dp* s = c->srv;
  std::vector<std::vector<std::string>> crs;
  if (!parse_allocate((const uint8_t*)body.data(), (const uint8_t*)body.data() + body.size(), &crs) ||
      crs.size() != 1 || crs[0].empty()) {
    s->n.shape++;
    return false;
  }
  int64_t l0 = mono_ns();
  std::unique_lock<std::mutex> lk(s->mu);
  int64_t l1 = mono_ns();
  if (!s->table.valid) {                    // no table (the engine serves every Allocate itself)
    s->n.stale++;
    return false;
  }
  uint64_t tw = 0, ww = 0;
  if (!table_current(s)) {
    // the pod cache or the engine moved since the table was built: the engine republishes
    // within a few hundred microseconds (its prepare loop wakes on the same change)
    s->n.waited++;
    int64_t w0 = mono_ns();
    wait_for_table(s, lk, s->fast_wait_us, [&] { return table_current(s) || s->blocked > 0 || s->stopping.load(); });
    tw = (uint64_t)(mono_ns() - w0);
    s->n.wait_ns += tw;
    if (!table_current(s)) {
      (s->blocked > 0 ? s->n.blocked : s->n.stale)++;
      return false;
    }
  }
  const Entry* en = nullptr;
  Decline d = pick(s, crs[0], &en);
  if (d == kNoMatch && s->watch_wait_us > 0) {
    // no candidate of this size yet: the kubelet's own pod watch can deliver the bind before
    // the plugin's does; the engine's cache hook publishes the pod the moment it arrives, so
    // wait for the next table (a LIST on the engine's path is the alternative)
    // (a pre-bind entry is published at the same cache version: any new table counts)
    s->n.watch_waits++;
    int64_t w0 = mono_ns(), dl = w0 + (int64_t)s->watch_wait_us * 1000;
    while (d == kNoMatch) {
      int left_us = (int)((dl - mono_ns()) / 1000);
      if (left_us <= 0) break;
      uint64_t seq = s->pub_seq;
      wait_for_table(s, lk, left_us, [&] {
        return (s->pub_seq != seq && table_current(s)) || s->blocked > 0 || s->stopping.load();
      });
      if (s->blocked > 0 || s->stopping.load() || !table_current(s)) break;
      if (s->pub_seq != seq) d = pick(s, crs[0], &en);
    }
    ww = (uint64_t)(mono_ns() - w0);
  }
  if (d != kOk) {
    count_decline(s, d);
    return false;
  }
  double t = wall_s();
  int64_t j0 = mono_ns();
  if (!journal_append(s, *en, body, t)) {  // journal before the reply
    s->n.journal++;
    return false;
  }
  int64_t j1 = mono_ns();
  const_cast<Entry*>(en)->taken = true;
  s->taken_uids.insert(en->uid);
  for (auto& id : crs[0]) s->answered_ids[id] = t_in;
  uint64_t hns = (uint64_t)(mono_ns() - t_in);
  s->taken.push_back(Taken{en->uid, body, t, hns, t_in, ww, tw});
  std::string resp = en->body;
  s->n.fast++;
  s->n.lock_ns += (uint64_t)(l1 - l0);
  s->n.journal_ns += (uint64_t)(j1 - j0);
  s->n.answer_ns += (uint64_t)(mono_ns() - t_in);
  lk.unlock();
  // the engine's claim reader is woken once the reply is on the wire (serve_conn): its
  // bookkeeping and the write-behind PATCH it starts must not compete with the reply
  c->wake_taken = true;
  respond(c, sid, 0, "", resp, true);
  return true;
}

// ---- request dispatch -------------------------------------------------------------------
const char* kAllocate = "/v1beta1.DevicePlugin/Allocate";
const char* kLaW = "/v1beta1.DevicePlugin/ListAndWatch";
const char* kForward[] = {"/v1beta1.DevicePlugin/GetDevicePluginOptions", "/v1beta1.DevicePlugin/PreStartContainer",
                          "/v1beta1.DevicePlugin/GetPreferredAllocation", kAllocate};

void start_law(Conn* c, int32_t sid) {
  gs_dp* s = c->srv;
  Stream& st = c->streams[sid];
  st.law = true;
  {
    std::lock_guard<std::mutex> lk(s->dev_mu);
    st.out = s->devices;
    c->sent_dev_gen = std::max(c->sent_dev_gen, s->dev_gen);
  }
  st.off = 0;
  s->n.law_sends++;
  nghttp2_nv h[] = {nv(":status", kStatus200), nv("content-type", kCtype)};
  nghttp2_data_provider dp;
  dp.source.ptr = nullptr;
  dp.read_callback = read_cb;
  nghttp2_submit_response(c->sess, sid, h, 2, &dp);
}

void request_done(Conn* c, int32_t sid) {
  gs_dp* s = c->srv;
  auto it = c->streams.find(sid);
  if (it == c->streams.end()) return;
  Stream& st = it->second;
  st.t_in = mono_ns();
  const std::string& b = st.body;
  if (st.too_big) {
    respond(c, sid, 8, "request larger than " + std::to_string(kMaxRequest - 5) + " bytes", "", false);
    return;
  }
  if (b.size() < 5 || b[0] != 0) {
    respond(c, sid, b.size() >= 5 ? 12 : 13, b.size() >= 5 ? "compressed messages are not supported"
                                                            : "malformed gRPC message", "", false);
    return;
  }
  uint32_t len = (uint8_t)b[1] << 24 | (uint8_t)b[2] << 16 | (uint8_t)b[3] << 8 | (uint8_t)b[4];
  if (len != b.size() - 5) {
    respond(c, sid, 13, "malformed gRPC message length", "", false);
    return;
  }
  std::string msg = b.substr(5);
  if (st.path == kLaW) {
    start_law(c, sid);
    return;
  }
  bool known = false;
  for (const char* m : kForward) known |= st.path == m;
  if (!known) {
    s->n.unknown++;
    respond(c, sid, 12, "unknown method " + st.path, "", false);
    return;
  }
  if (st.path == kAllocate) {
    if (fast_allocate(c, sid, msg, st.t_in)) return;
    s->n.forwarded_allocate++;
  }
  auto f = std::make_shared<Fwd>();
  f->conn = c->self;
  f->stream = sid;
  f->method = st.path;
  f->body = std::move(msg);
  f->t_in = st.t_in;
  f->deadline = st.deadline;
  {
    std::lock_guard<std::mutex> lk(s->q_mu);
    f->id = s->next_id++;
    s->queue.push_back(f);
  }
  s->n.forwarded++;
  s->q_cv.notify_one();
}

// ---- nghttp2 callbacks ------------------------------------------------------------------
int on_begin_headers(nghttp2_session*, const nghttp2_frame* f, void* ud) {
  if (f->hd.type == NGHTTP2_HEADERS && f->headers.cat == NGHTTP2_HCAT_REQUEST)
    static_cast<Conn*>(ud)->streams[f->hd.stream_id];
  return 0;
}

int on_header(nghttp2_session*, const nghttp2_frame* f, const uint8_t* name, size_t nl, const uint8_t* value,
              size_t vl, uint8_t, void* ud) {
  if (f->hd.type != NGHTTP2_HEADERS || f->headers.cat != NGHTTP2_HCAT_REQUEST) return 0;
  if (nl == 5 && !memcmp(name, ":path", 5)) {
    auto it = static_cast<Conn*>(ud)->streams.find(f->hd.stream_id);
    if (it != static_cast<Conn*>(ud)->streams.end()) it->second.path.assign((const char*)value, vl);
  } else if (nl == 12 && !memcmp(name, "grpc-timeout", 12)) {
    auto it = static_cast<Conn*>(ud)->streams.find(f->hd.stream_id);
    int64_t t = parse_grpc_timeout_ns(value, vl);
    if (it != static_cast<Conn*>(ud)->streams.end() && t > 0) it->second.deadline = mono_ns() + t;
  }
  return 0;
}

int on_data_chunk(nghttp2_session*, uint8_t, int32_t sid, const uint8_t* d, size_t l, void* ud) {
  Conn* c = static_cast<Conn*>(ud);
  auto it = c->streams.find(sid);
  if (it == c->streams.end()) return 0;
  Stream& st = it->second;
  if (st.too_big || st.body.size() + l > kMaxRequest) {
    st.too_big = true;
    std::string().swap(st.body);
    return 0;
  }
  st.body.append((const char*)d, l);
  return 0;
}

int on_frame_recv(nghttp2_session*, const nghttp2_frame* f, void* ud) {
  if ((f->hd.type == NGHTTP2_DATA || f->hd.type == NGHTTP2_HEADERS) && (f->hd.flags & NGHTTP2_FLAG_END_STREAM))
    request_done(static_cast<Conn*>(ud), f->hd.stream_id);
  return 0;
}

int on_stream_close(nghttp2_session*, int32_t sid, uint32_t, void* ud) {
  static_cast<Conn*>(ud)->streams.erase(sid);
  return 0;
}

bool write_all(int fd, const uint8_t* p, size_t n) {
  while (n) {
    ssize_t w = send(fd, p, n, MSG_NOSIGNAL);
    if (w < 0) {
      if (errno == EINTR) continue;
      return false;
    }
    p += w;
    n -= (size_t)w;
  }
  return true;
}

void drain_outbox(Conn* c) {
  gs_dp* s = c->srv;
  std::vector<Reply> out;
  {
    std::lock_guard<std::mutex> lk(c->out_mu);
    out.swap(c->outbox);
  }
  for (auto& r : out) respond(c, r.stream, r.status, r.message, r.body, true);
  uint64_t g;
  std::string dev;
  {
    std::lock_guard<std::mutex> lk(s->dev_mu);
    g = s->dev_gen;
    if (g != c->sent_dev_gen) dev = s->devices;
  }
  if (g != c->sent_dev_gen) {
    c->sent_dev_gen = g;
    for (auto& kv : c->streams) {
      if (!kv.second.law) continue;
      kv.second.out += dev;
      s->n.law_sends++;
      nghttp2_session_resume_data(c->sess, kv.first);
    }
  }
}

void serve_conn(std::shared_ptr<Conn> cp) {
  Conn* c = cp.get();
  nghttp2_session_callbacks* cb;
  nghttp2_session_callbacks_new(&cb);
  nghttp2_session_callbacks_set_on_begin_headers_callback(cb, on_begin_headers);
  nghttp2_session_callbacks_set_on_header_callback(cb, on_header);
  nghttp2_session_callbacks_set_on_data_chunk_recv_callback(cb, on_data_chunk);
  nghttp2_session_callbacks_set_on_frame_recv_callback(cb, on_frame_recv);
  nghttp2_session_callbacks_set_on_stream_close_callback(cb, on_stream_close);
  nghttp2_session_server_new(&c->sess, cb, c);
  nghttp2_session_callbacks_del(cb);
  nghttp2_settings_entry iv[] = {{NGHTTP2_SETTINGS_MAX_CONCURRENT_STREAMS, 256},
                                 {NGHTTP2_SETTINGS_INITIAL_WINDOW_SIZE, 1u << 20}};
  nghttp2_submit_settings(c->sess, NGHTTP2_FLAG_NONE, iv, 2);
  nghttp2_session_set_local_window_size(c->sess, NGHTTP2_FLAG_NONE, 0, 16 << 20);
  std::vector<uint8_t> buf(1 << 16);
  std::string wbuf;
  bool term = false;
  for (;;) {
    // everything this turn produced goes out in one write: a reply's HEADERS, DATA and
    // trailers arriving as separate writes wake the client's poller once per frame
    const uint8_t* data;
    ssize_t n;
    wbuf.clear();
    while ((n = nghttp2_session_mem_send(c->sess, &data)) > 0) wbuf.append((const char*)data, (size_t)n);
    if (!wbuf.empty() && !write_all(c->fd, (const uint8_t*)wbuf.data(), wbuf.size())) break;
    if (c->wake_taken) {
      c->wake_taken = false;
      std::lock_guard<std::mutex> lk(c->srv->mu);   // pairs with gs_dp_taken_next's wait
      c->srv->taken_cv.notify_all();
    }
    if (n < 0) break;
    if (!nghttp2_session_want_read(c->sess) && !nghttp2_session_want_write(c->sess)) break;
    pollfd fds[2] = {{c->fd, POLLIN, 0}, {c->efd, POLLIN, 0}};
    bool spin = c->srv->spin_until.load(std::memory_order_relaxed) > mono_ns();
    int pr = poll(fds, 2, spin ? 0 : -1);
    if (pr < 0) {
      if (errno == EINTR) continue;
      break;
    }
    if (pr == 0) {                             // spinning, nothing yet
      // yield, not pause: a thread that shares this CPU (the kubelet's, the plugin's pod
      // watch) must run at once, not after a scheduler time slice (~ms) of our spinning
      sched_yield();
      continue;
    }
    if (fds[1].revents & POLLIN) {
      uint64_t v;
      ssize_t r = read(c->efd, &v, sizeof v);
      (void)r;
      if (c->srv->stopping.load() && !term) {
        term = true;
        c->closing.store(true);
        for (auto& kv : c->streams)
          if (kv.second.law) nghttp2_session_resume_data(c->sess, kv.first);   // end the streams
        nghttp2_session_terminate_session(c->sess, NGHTTP2_NO_ERROR);
      }
      drain_outbox(c);
    }
    if (fds[0].revents & (POLLIN | POLLHUP | POLLERR)) {
      ssize_t r = recv(c->fd, buf.data(), buf.size(), 0);
      if (r <= 0) {
        if (r < 0 && errno == EINTR) continue;
        break;
      }
      if (nghttp2_session_mem_recv(c->sess, buf.data(), (size_t)r) < 0) break;
    }
  }
  nghttp2_session_del(c->sess);
  c->sess = nullptr;
  c->streams.clear();
  close(c->fd);
  c->done.store(true);
}

void accept_loop(gs_dp* s) {
  while (!s->stopping.load()) {
    int fd = accept4(s->lfd, nullptr, nullptr, SOCK_CLOEXEC);
    if (fd < 0) {
      if (errno == EINTR || errno == ECONNABORTED) continue;
      break;
    }
    if (s->stopping.load()) {
      close(fd);
      break;
    }
    auto c = std::make_shared<Conn>();
    c->srv = s;
    c->fd = fd;
    c->self = c;
    c->efd = eventfd(0, EFD_CLOEXEC | EFD_NONBLOCK);
    if (c->efd < 0) {
      close(fd);
      continue;
    }
    s->n.conns++;
    std::lock_guard<std::mutex> lk(s->conns_mu);
    // connections that ended are joined and dropped (a client that reconnects over and over
    // costs nothing that stays); the eventfd goes with the last reference
    std::vector<std::shared_ptr<Conn>> live;
    for (auto& x : s->conns) {
      if (x->done.load()) {
        if (x->th.joinable()) x->th.join();
      } else {
        live.push_back(x);
      }
    }
    c->th = std::thread(serve_conn, c);
    live.push_back(c);
    s->conns.swap(live);
  }
}

void set_err(char* err, int errlen, const char* fmt, ...) {
  if (!err || errlen <= 0) return;
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(err, (size_t)errlen, fmt, ap);
  va_end(ap);
}

}  // namespace

extern "C" {

gs_dp* gs_dp_start(const char* socket_path, char* err, int errlen) {
  sockaddr_un a{};
  if (strlen(socket_path) >= sizeof a.sun_path) {
    set_err(err, errlen, "socket path too long: %s", socket_path);
    return nullptr;
  }
  int fd = socket(AF_UNIX, SOCK_STREAM | SOCK_CLOEXEC, 0);
  if (fd < 0) {
    set_err(err, errlen, "socket: %s", strerror(errno));
    return nullptr;
  }
  a.sun_family = AF_UNIX;
  strcpy(a.sun_path, socket_path);
  unlink(socket_path);
  if (bind(fd, (sockaddr*)&a, sizeof a) != 0 || listen(fd, 64) != 0) {
    set_err(err, errlen, "listen on %s: %s", socket_path, strerror(errno));
    close(fd);
    return nullptr;
  }
  auto* s = new gs_dp();
  s->path = socket_path;
  s->lfd = fd;
  s->acceptor = std::thread(accept_loop, s);
  return s;
}

void gs_dp_stop(gs_dp* s) {
  if (!s) return;
  s->stopping.store(true);
  shutdown(s->lfd, SHUT_RDWR);
  close(s->lfd);
  if (s->acceptor.joinable()) s->acceptor.join();
  std::vector<std::shared_ptr<Conn>> conns;
  {
    std::lock_guard<std::mutex> lk(s->conns_mu);
    conns.swap(s->conns);
  }
  for (auto& c : conns) wake(c.get());
  for (auto& c : conns)
    if (c->th.joinable()) c->th.join();
  conns.clear();
  s->q_cv.notify_all();
  {
    std::lock_guard<std::mutex> lk(s->mu);
    s->cv.notify_all();
  }
  s->taken_cv.notify_all();
  unlink(s->path.c_str());
  // the handle itself stays allocated: Python threads may still be returning from
  // gs_dp_next / gs_dp_taken_next (they see -1); the journal mapping is released here
  std::lock_guard<std::mutex> lk(s->mu);
  if (s->jmap) munmap(s->jmap, s->jsize), s->jmap = nullptr;
  if (s->jfd >= 0) close(s->jfd), s->jfd = -1;
  s->table = Table();
  s->answered_ids.clear();
  s->taken_uids.clear();
}

int64_t gs_dp_next(gs_dp* s, int timeout_ms, char* method, int method_cap, uint8_t* body, int body_cap,
                   int* body_len, int64_t* t_in_ns) {
  for (;;) {
    std::shared_ptr<Fwd> f;
    {
      std::unique_lock<std::mutex> lk(s->q_mu);
      if (!s->q_cv.wait_until(lk, deadline_us(1000LL * timeout_ms),
                              [&] { return !s->queue.empty() || s->stopping.load(); }))
        return 0;
      if (s->stopping.load()) return -1;
      f = s->queue.front();
      s->queue.pop_front();
      if ((int)f->body.size() <= body_cap && (int)f->method.size() < method_cap) s->inflight[f->id] = f;
    }
    if (f->deadline && mono_ns() > f->deadline) {
      // the client gave up while the request waited for a handler (the kubelet's admission of
      // that pod already failed): running it would only claim a pod for nobody
      {
        std::lock_guard<std::mutex> lk(s->q_mu);
        s->inflight.erase(f->id);
      }
      s->n.expired++;
      if (auto c = f->conn.lock()) {
        {
          std::lock_guard<std::mutex> lk(c->out_mu);
          c->outbox.push_back(Reply{f->stream, 4, "deadline exceeded before a handler took the request", ""});
        }
        wake(c.get());
      }
      continue;
    }
    if ((int)f->body.size() > body_cap || (int)f->method.size() >= method_cap) {
      if (auto c = f->conn.lock()) {
        {
          std::lock_guard<std::mutex> lk(c->out_mu);
          c->outbox.push_back(Reply{f->stream, 8, "request too large", ""});
        }
        wake(c.get());
      }
      continue;
    }
    memcpy(method, f->method.c_str(), f->method.size() + 1);
    memcpy(body, f->body.data(), f->body.size());
    *body_len = (int)f->body.size();
    *t_in_ns = f->t_in;
    return f->id;
  }
}

int gs_dp_reply(gs_dp* s, int64_t id, int grpc_status, const char* message, const uint8_t* body, int body_len) {
  std::shared_ptr<Fwd> f;
  {
    std::lock_guard<std::mutex> lk(s->q_mu);
    auto it = s->inflight.find(id);
    if (it == s->inflight.end()) return -1;
    f = it->second;
    s->inflight.erase(it);
  }
  auto c = f->conn.lock();
  if (!c) return -1;
  {
    std::lock_guard<std::mutex> lk(c->out_mu);
    c->outbox.push_back(Reply{f->stream, grpc_status, message ? message : "",
                              body ? std::string((const char*)body, (size_t)body_len) : std::string()});
  }
  wake(c.get());
  return 0;
}

int gs_dp_set_devices(gs_dp* s, const uint8_t* body, int len) {
  {
    std::lock_guard<std::mutex> lk(s->dev_mu);
    s->devices = grpc_frame(std::string((const char*)body, (size_t)len));
    s->dev_gen++;
  }
  std::lock_guard<std::mutex> lk(s->conns_mu);
  for (auto& c : s->conns)
    if (!c->done.load()) wake(c.get());
  return 0;
}

int gs_dp_fast_publish(gs_dp* s, const uint8_t* blob, int len) {
  Table t;
  if (!parse_table(blob, len, &t)) return -1;
  t.valid = !(t.flags & 0x80000000u);       // flag 31: no table (fast path off)
  {
    std::lock_guard<std::mutex> lk(s->mu);
    // two publishers (the engine's prepare loop and its pod-cache hook) may finish out of
    // order: a table older than the one held is dropped, never installed over it
    if (t.valid && s->table.valid &&
        (t.gen < s->table.gen || (t.gen == s->table.gen && t.version < s->table.version))) {
      s->n.older++;
      return 0;
    }
    // A claim stays a claim while the new table still lists the pod (the engine built it
    // before it processed the claim) or the engine has not taken the claim's record yet.
    std::unordered_set<std::string> keep;
    for (auto& tk : s->taken) keep.insert(tk.uid);
    for (auto& en : t.entries)
      if (s->taken_uids.count(en.uid)) keep.insert(en.uid);
    s->taken_uids.swap(keep);
    for (auto& en : t.entries) en.taken = s->taken_uids.count(en.uid) > 0;
    int64_t now = mono_ns();
    for (auto it = s->answered_ids.begin(); it != s->answered_ids.end();)
      it = (t.replay.count(it->first) || now - it->second > 30 * 1000000000LL) ? s->answered_ids.erase(it) : ++it;
    s->table = std::move(t);
    s->table_seq++;
    s->pub_seq++;
  }
  s->cv.notify_all();
  return 0;
}

void gs_dp_set_version(gs_dp* s, uint64_t version) {
  {
    std::lock_guard<std::mutex> lk(s->mu);
    s->cur_version = std::max(s->cur_version, version);   // versions only grow
    s->table_seq++;
  }
  s->cv.notify_all();
}

void gs_dp_set_gen(gs_dp* s, uint64_t gen) {
  {
    std::lock_guard<std::mutex> lk(s->mu);
    s->cur_gen = std::max(s->cur_gen, gen);
    s->table_seq++;
  }
  s->cv.notify_all();
}

void gs_dp_fast_block(gs_dp* s) {
  {
    std::lock_guard<std::mutex> lk(s->mu);   // an answer in progress holds mu: it completes first
    s->blocked++;
    s->table_seq++;
  }
  s->cv.notify_all();
}

void gs_dp_fast_unblock(gs_dp* s) {
  {
    std::lock_guard<std::mutex> lk(s->mu);
    if (s->blocked > 0) s->blocked--;
    s->table_seq++;
  }
  s->cv.notify_all();
}

void gs_dp_fast_take(gs_dp* s, const char* uid) {
  std::lock_guard<std::mutex> lk(s->mu);
  s->taken_uids.insert(uid);
  for (auto& en : s->table.entries)
    if (en.uid == uid) en.taken = true;
}

void gs_dp_set_fast_wait_us(gs_dp* s, int us) {
  std::lock_guard<std::mutex> lk(s->mu);
  s->fast_wait_us = us < 0 ? 0 : us;
}

void gs_dp_spin(gs_dp* s, int us) {
  int64_t until = mono_ns() + (int64_t)us * 1000;
  int64_t cur = s->spin_until.load();
  while (until > cur && !s->spin_until.compare_exchange_weak(cur, until)) {
  }
  std::lock_guard<std::mutex> lk(s->conns_mu);
  for (auto& c : s->conns)
    if (!c->done.load()) wake(c.get());      // out of a sleeping poll, into the spin
}

void gs_dp_set_watch_wait_us(gs_dp* s, int us) {
  std::lock_guard<std::mutex> lk(s->mu);
  s->watch_wait_us = us < 0 ? 0 : us;
}

int gs_dp_taken_next(gs_dp* s, int timeout_ms, uint8_t* buf, int cap) {
  std::unique_lock<std::mutex> lk(s->mu);
  if (!s->taken_cv.wait_until(lk, deadline_us(1000LL * timeout_ms),
                              [&] { return !s->taken.empty() || s->stopping.load(); }))
    return 0;
  if (s->taken.empty()) return -1;
  const Taken& t = s->taken.front();
  size_t need = 4 + t.uid.size() + 4 + t.req.size() + 8 + 8 + 24;
  if ((size_t)cap < need) return -2;
  uint8_t* p = buf;
  uint32_t l = (uint32_t)t.uid.size();
  memcpy(p, &l, 4), p += 4;
  memcpy(p, t.uid.data(), l), p += l;
  l = (uint32_t)t.req.size();
  memcpy(p, &l, 4), p += 4;
  memcpy(p, t.req.data(), l), p += l;
  memcpy(p, &t.t, 8), p += 8;
  memcpy(p, &t.handler_ns, 8), p += 8;
  memcpy(p, &t.t_in, 8), p += 8;
  memcpy(p, &t.watch_wait_ns, 8), p += 8;
  memcpy(p, &t.table_wait_ns, 8), p += 8;
  // the engine now knows the claim; the uid stays in taken_uids (the table entry must not be
  // answered again) until the next publish no longer lists it
  s->taken.pop_front();
  return (int)need;
}

int gs_dp_taken_pending(gs_dp* s) {
  std::lock_guard<std::mutex> lk(s->mu);
  return (int)s->taken.size();
}

int gs_dp_fast_journal_open(gs_dp* s, const char* path, uint64_t bytes) {
  int fd = open(path, O_RDWR | O_CREAT | O_CLOEXEC, 0600);
  if (fd < 0) return -1;
  struct stat st;
  if (fstat(fd, &st) != 0) return close(fd), -1;
  uint64_t size = std::max<uint64_t>(bytes, (uint64_t)st.st_size);
  if (ftruncate(fd, (off_t)size) != 0) return close(fd), -1;
  posix_fallocate(fd, 0, (off_t)size);
  void* m = mmap(nullptr, size, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
  if (m == MAP_FAILED) return close(fd), -1;
  auto* p = static_cast<uint8_t*>(m);
  uint64_t end = 0;
  while (end < size && p[end]) ++end;          // records end at the first zero byte
  // fault the pages in, writable, now: a plain p[o] = p[o] is a no-op the compiler removes,
  // and then every first append to a page paid a write fault (~40 us) on the Allocate path
  volatile uint8_t* vp = p;
  for (uint64_t o = end - end % 4096; o < size; o += 4096) vp[o] = vp[o];
  std::lock_guard<std::mutex> lk(s->mu);
  if (s->jmap) munmap(s->jmap, s->jsize);
  if (s->jfd >= 0) close(s->jfd);
  s->jfd = fd;
  s->jmap = p;
  s->jsize = size;
  s->joff = end;
  return 0;
}

// Re-dirty the pages the next appends will write (the current one and the two after it):
// writeback cleans a page (and write-protects its mapping) ~30 s after it was dirtied, and the
// next append would take the write fault. The engine calls this off the Allocate path.
void gs_dp_fast_journal_prefault(gs_dp* s) {
  std::lock_guard<std::mutex> lk(s->mu);
  if (!s->jmap) return;
  volatile uint8_t* vp = s->jmap;
  for (uint64_t o = s->joff - s->joff % 4096, n = 0; o < s->jsize && n < 3; o += 4096, ++n) vp[o] = vp[o];
}

uint64_t gs_dp_fast_journal_used(gs_dp* s) {
  std::lock_guard<std::mutex> lk(s->mu);
  return s->joff;
}

int gs_dp_fast_journal_rotate(gs_dp* s) {
  std::lock_guard<std::mutex> lk(s->mu);
  if (!s->jmap) return -1;
  memset(s->jmap, 0, s->joff);
  s->joff = 0;
  return 0;
}

int gs_dp_stats(gs_dp* s, char* buf, int cap) {
  uint64_t used, pend;
  {
    std::lock_guard<std::mutex> lk(s->mu);
    used = s->joff;
    pend = s->taken.size();
  }
  int n = snprintf(buf, (size_t)cap,
                   "{\"fast\":%llu,\"forwarded\":%llu,\"forwarded_allocate\":%llu,\"declined\":{\"stale\":%llu,\"blocked\":%llu,\"replay\":%llu,"
                   "\"nomatch\":%llu,\"multi\":%llu,\"ambiguous\":%llu,\"shape\":%llu,\"journal\":%llu},"
                   "\"waited\":%llu,\"law_sends\":%llu,\"connections\":%llu,\"unknown\":%llu,\"older_tables\":%llu,\"expired\":%llu,\"watch_waits\":%llu,\"wait_ns\":%llu,\"lock_ns\":%llu,\"journal_ns\":%llu,\"answer_ns\":%llu,"
                   "\"journal_used\":%llu,\"taken_pending\":%llu}",
                   (unsigned long long)s->n.fast, (unsigned long long)s->n.forwarded,
                   (unsigned long long)s->n.forwarded_allocate, (unsigned long long)s->n.stale,
                   (unsigned long long)s->n.blocked, (unsigned long long)s->n.replay, (unsigned long long)s->n.nomatch,
                   (unsigned long long)s->n.multi, (unsigned long long)s->n.ambiguous, (unsigned long long)s->n.shape,
                   (unsigned long long)s->n.journal, (unsigned long long)s->n.waited,
                   (unsigned long long)s->n.law_sends, (unsigned long long)s->n.conns,
                   (unsigned long long)s->n.unknown, (unsigned long long)s->n.older, (unsigned long long)s->n.expired, (unsigned long long)s->n.watch_waits,
                   (unsigned long long)s->n.wait_ns, (unsigned long long)s->n.lock_ns,
                   (unsigned long long)s->n.journal_ns, (unsigned long long)s->n.answer_ns, (unsigned long long)used,
                   (unsigned long long)pend);
  return n < cap ? n : -1;
}

}  // extern "C"
