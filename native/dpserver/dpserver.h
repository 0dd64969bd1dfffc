// libgpushare_dpserver.so — the kubelet DevicePlugin gRPC service served natively (C ABI).
//
// gRPC over HTTP/2 on the plugin's Unix socket (nghttp2 for the framing, HPACK and flow
// control), with the common Allocate answered in this library: the Python engine publishes
// its prepared answers (one per candidate pod, in match order) and the library picks, claims,
// journals and replies without entering the interpreter. Everything else — the other RPCs
// and every Allocate the fast table cannot answer exactly as the engine would — is handed to
// Python handler threads (gs_dp_next / gs_dp_reply), and ListAndWatch is streamed from the
// device list Python sets (gs_dp_set_devices). See plugin/native_server.py.
#pragma once
#include <stddef.h>
#include <stdint.h>

#define GS_DP_API __attribute__((visibility("default")))

#ifdef __cplusplus
extern "C" {
#endif

typedef struct gs_dp gs_dp;

// Listen on `socket_path` (an existing file there is removed). NULL on error (message in err).
GS_DP_API gs_dp* gs_dp_start(const char* socket_path, char* err, int errlen);
// Stop serving: GOAWAY to every connection, wake every waiter, join the threads, remove the socket.
GS_DP_API void gs_dp_stop(gs_dp* s);

// Next request for Python. Returns its id (> 0), 0 on timeout, -1 once stopped. The method
// path goes to `method` (NUL-terminated), the request message to `body` (*body_len bytes);
// *t_in_ns is when the request was complete (CLOCK_MONOTONIC). A body larger than body_cap is
// answered RESOURCE_EXHAUSTED here and never returned.
GS_DP_API int64_t gs_dp_next(gs_dp* s, int timeout_ms, char* method, int method_cap, uint8_t* body, int body_cap,
                   int* body_len, int64_t* t_in_ns);
// Answer request `id`: grpc_status 0 with the serialized response, or an error status + message.
GS_DP_API int gs_dp_reply(gs_dp* s, int64_t id, int grpc_status, const char* message, const uint8_t* body, int body_len);

// ListAndWatch: the serialized ListAndWatchResponse every stream sends now and after each change.
GS_DP_API int gs_dp_set_devices(gs_dp* s, const uint8_t* body, int len);

// ---- Allocate fast path ------------------------------------------------------------------
// The table (see dpserver.cpp "table blob") carries the cache version and engine generation
// it was built at; answers are given only while both still match gs_dp_set_version/_gen.
GS_DP_API int gs_dp_fast_publish(gs_dp* s, const uint8_t* blob, int len);
GS_DP_API void gs_dp_set_version(gs_dp* s, uint64_t version);
GS_DP_API void gs_dp_set_gen(gs_dp* s, uint64_t gen);
// Block / unblock native answers (counted). Block returns once no native answer is in progress.
GS_DP_API void gs_dp_fast_block(gs_dp* s);
GS_DP_API void gs_dp_fast_unblock(gs_dp* s);
// The engine claimed pod `uid` itself: never answer it from the table.
GS_DP_API void gs_dp_fast_take(gs_dp* s, const char* uid);
// How long an Allocate may wait for a table matching the current version/generation.
GS_DP_API void gs_dp_set_fast_wait_us(gs_dp* s, int us);
// How long an Allocate no candidate matches may wait for the pod watch (a newer table) before
// it goes to the engine.
GS_DP_API void gs_dp_set_watch_wait_us(gs_dp* s, int us);
// Busy-poll the kubelet connections for the next `us` microseconds (an Allocate is expected:
// a pod was just published) instead of sleeping in poll.
GS_DP_API void gs_dp_spin(gs_dp* s, int us);
// Next native answer for the engine's bookkeeping: record = u32 uid_len, uid, u32 req_len,
// AllocateRequest bytes, f64 wall time (the journal record's "t"), u64 handler ns. Returns the
// record size, 0 on timeout, -1 once stopped, -2 if `cap` is too small (record kept).
GS_DP_API int gs_dp_taken_next(gs_dp* s, int timeout_ms, uint8_t* buf, int cap);
GS_DP_API int gs_dp_taken_pending(gs_dp* s);
// The native answers' journal (same JSON-lines records as the engine's fast path, written
// before the reply): a pre-sized file, mapped; rotate = zero it after the engine compacted
// its own journal with everything in it.
GS_DP_API int gs_dp_fast_journal_open(gs_dp* s, const char* path, uint64_t bytes);
GS_DP_API uint64_t gs_dp_fast_journal_used(gs_dp* s);
// Re-dirty the next pages the journal appends will write (off the Allocate path).
GS_DP_API void gs_dp_fast_journal_prefault(gs_dp* s);
GS_DP_API int gs_dp_fast_journal_rotate(gs_dp* s);

// Counters as a JSON object (NUL-terminated); returns its length or -1.
GS_DP_API int gs_dp_stats(gs_dp* s, char* buf, int cap);

// ---- gRPC unary client (h2client.cpp): the simulated kubelet's device-manager calls ---------
typedef struct gs_h2c gs_h2c;
GS_DP_API gs_h2c* gs_h2c_connect(const char* socket_path);
GS_DP_API int gs_h2c_unary(gs_h2c* h, const char* path, const uint8_t* req, int len, uint8_t* out, int cap,
                           int* out_len, int* status, char* message, int mcap, char* stamp, int scap,
                           int timeout_ms, int64_t* t_send, int64_t* t_recv);
// gs_h2c_unary with the DATA payload sent as given (no gRPC length prefix added).
GS_DP_API int gs_h2c_call(gs_h2c* h, const char* path, const uint8_t* body, int len, uint8_t* out, int cap,
                          int* out_len, int* status, char* message, int mcap, char* stamp, int scap,
                          int timeout_ms, int64_t* t_send, int64_t* t_recv);
GS_DP_API void gs_h2c_close(gs_h2c* h);

#ifdef __cplusplus
}
#endif
