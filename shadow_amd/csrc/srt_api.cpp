// srt_api.cpp -- host side of the MI355X routing-table build: the C ABI of
// include/srt.h, plan lifetime, validation and the key-representation choice.
//
// Mirrors the reference call sequence of NetworkGraph::compute_shortest_paths
// (src/main/network/graph/mod.rs:183-228):
//   1. shortest paths between in-use nodes (here: device kernels);
//   2. diagonal := the unique self-loop edge, else "No edge connecting node X
//      to X" / "More than one edge connecting node X to X" (mod.rs:210-217,
//      256-293) -- validated on the host before any device work, in node order;
//   3. every ordered pair must be reachable (the assert at mod.rs:219) ->
//      SRT_ERR_DISCONNECTED.
#include <hip/hip_runtime.h>
#include <immintrin.h>
#include <sys/mman.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <atomic>
#include <condition_variable>
#include <deque>
#include <cstring>
#include <memory>
#include <mutex>
#include <new>
#include <numeric>
#include <string>
#include <queue>
#include <thread>
#include <vector>

#include "srt_internal.h"
#include "srt_scan.h"

using srt::CsrStats;
using srt::KeyParams;
using srt::csr_scan;
using srt::host_threads;
using srt::merge_stats;
using srt::scan_rows;

namespace {

void set_err(srt_err *err, int code, const char *msg, uint32_t a = 0, uint32_t b = 0) {
    if (!err) return;
    err->code = code;
    err->a_id = a;
    err->b_id = b;
    std::snprintf(err->msg, sizeof err->msg, "%s", msg);
}

void clear_err(srt_err *err) {
    if (err) std::memset(err, 0, sizeof *err);
}

srt_status build_loss_rows(srt_plan *p, int W, uint32_t rows_per, srt_err *err);

srt_status hip_fail(srt_err *err, hipError_t e, const char *what) {
    char buf[256];
    std::snprintf(buf, sizeof buf, "%s: %s", what, hipGetErrorString(e));
    set_err(err, SRT_ERR_HIP, buf);
    return e == hipErrorOutOfMemory ? SRT_ERR_OOM : SRT_ERR_HIP;
}

#define HIP_TRY(expr, what)                                \
    do {                                                   \
        hipError_t e_ = (expr);                            \
        if (e_ != hipSuccess) return hip_fail(err, e_, what); \
    } while (0)

uint32_t node_id(const srt_csr *g, uint32_t idx) { return g->node_ids ? g->node_ids[idx] : idx; }

// SRT_TRACE=1: host-side phase timings on stderr (measurement only)
struct Trace {
    bool on = std::getenv("SRT_TRACE") != nullptr;
    std::chrono::steady_clock::time_point t0 = std::chrono::steady_clock::now(), last = t0;
    void mark(const char *what) {
        if (!on) return;
        const auto now = std::chrono::steady_clock::now();
        std::fprintf(stderr, "[srt] %-28s %9.3f ms (total %9.3f)\n", what,
                     std::chrono::duration<double, std::milli>(now - last).count(),
                     std::chrono::duration<double, std::milli>(now - t0).count());
        last = now;
    }
};

srt_status edge_error(srt_err *err, int c, uint32_t a_id, uint32_t b_id) {
    char buf[160];
    if (c == 0) {
        std::snprintf(buf, sizeof buf, "No edge connecting node %u to %u", a_id, b_id);
        set_err(err, SRT_ERR_NO_EDGE, buf, a_id, b_id);
        return SRT_ERR_NO_EDGE;
    }
    std::snprintf(buf, sizeof buf, "More than one edge connecting node %u to %u", a_id, b_id);
    set_err(err, SRT_ERR_MULTI_EDGE, buf, a_id, b_id);
    return SRT_ERR_MULTI_EDGE;
}

// Pinned host staging of the piece-pipelined upload and download, kept for
// the process (pinning 192 MB costs tens of milliseconds, more than the
// transfers it speeds up), one user at a time (a concurrent build takes the
// pageable / 16-byte paths).
struct PinnedPool {
    std::mutex m;
    void *buf = nullptr;
    size_t bytes = 0;
    bool ensure(size_t need) {  // call with m held
        if (bytes >= need) return true;
        if (buf) (void)hipHostFree(buf);
        buf = nullptr;
        bytes = 0;
        if (hipHostMalloc(&buf, need, 0) != hipSuccess) return false;
        bytes = need;
        return true;
    }
};
PinnedPool g_pinned;
constexpr size_t PINNED_BYTES = 3ull * (1ull << 23) * 8;  // 3 pieces of 8 Mi 8-byte records = 3 x 16 Mi u32

// Piece-pipelined CSR scan + upload (graphs of >= 16 Mi adjacency entries).
// The CSR scan's host threads walk the rows in pieces of <= 16 Mi entries,
// in order, and write each piece's latencies as u32 into a pinned slot (3 in
// flight); the main thread uploads a finished piece (64 MB instead of the
// 128 MB of u64) and a device kernel widens it into d_lat.  A piece whose
// rows are all exactly the entries 0 .. V-1 in order (a complete graph with
// self-loops, as Shadow's atlas graphs) uploads no col at all: a kernel writes
// it.  A piece with a latency >= 2^32 ns, or irregular rows, sends that array
// from the caller's memory as before.  C3 (16k complete): 3.2 GB -> 1.07 GB
// over PCIe.  Knob (tests): SRT_UPLOAD_PIECE=
// log2 entries per piece (also forces the pipeline on small graphs).
struct PieceUpload {
    static constexpr int DEPTH = 3;
    const srt_csr *g = nullptr;
    uint64_t PE = 1ull << 24;
    std::vector<uint32_t> cut;  // piece c = rows [cut[c], cut[c+1])
    uint32_t P = 0;
    int T = 1;
    std::vector<CsrStats> part;
    std::vector<uint8_t> over, ident;  // per (piece, thread)
    std::unique_ptr<std::atomic<int>[]> done;
    std::atomic<int> ready{-1};
    std::vector<std::thread> pool;
    std::unique_lock<std::mutex> lk;
    uint32_t *slot[DEPTH] = {};
    hipEvent_t ev[DEPTH] = {};
    bool on = false;
    bool check_loss = true;

    bool init(const srt_csr *g_, CsrStats *cs, bool check_loss_) {
        g = g_;
        check_loss = check_loss_;
        const char *pe = std::getenv("SRT_UPLOAD_PIECE");
        if (pe) PE = 1ull << std::max(4, std::min(24, std::atoi(pe)));
        else if (g->n_adj < PE) return false;
        const uint32_t V = g->n_nodes;
        cut.push_back(0);
        while (cut.back() < V) {
            const uint64_t k0 = g->row_ptr[cut.back()];
            uint32_t r = (uint32_t)(std::upper_bound(g->row_ptr + cut.back(), g->row_ptr + V + 1, k0 + PE) - g->row_ptr) - 1;
            if (r <= cut.back()) return false;  // one row larger than a piece
            cut.push_back(std::min(r, V));
        }
        P = (uint32_t)cut.size() - 1;
        // only when the pinned staging already exists: pinning it costs more
        // than the pipeline saves (srt_compute_shortest_paths allocates it
        // behind its first closure, for the download)
        lk = std::unique_lock<std::mutex>(g_pinned.m, std::try_to_lock);
        if (!lk.owns_lock() || g_pinned.bytes < std::max<size_t>(PINNED_BYTES, DEPTH * PE * 4)) return false;
        for (int i = 0; i < DEPTH; ++i) slot[i] = reinterpret_cast<uint32_t *>(g_pinned.buf) + (uint64_t)i * PE;
        cs->sl_cnt.assign(V, 0);
        cs->sl_first.assign(V, ~0ull);
        T = host_threads(g->n_adj);
        part.assign(T, CsrStats());
        over.assign((size_t)P * T, 0);
        ident.assign((size_t)P * T, 1);
        done.reset(new std::atomic<int>[P]);
        for (uint32_t c = 0; c < P; ++c) done[c].store(0);
        ready.store(std::min<int>(DEPTH, (int)P) - 1);
        for (int w = 0; w < T; ++w) pool.emplace_back([this, cs, w] { work(cs, w); });
        on = true;
        return true;
    }
    void work(CsrStats *cs, int w) {
        for (uint32_t c = 0; c < P; ++c) {
            while (ready.load(std::memory_order_acquire) < (int)c) std::this_thread::yield();
            const uint64_t k0 = g->row_ptr[cut[c]], k1 = g->row_ptr[cut[c + 1]];
            auto row_at = [&](uint64_t k) {
                return (uint32_t)(std::lower_bound(g->row_ptr + cut[c], g->row_ptr + cut[c + 1], k) - g->row_ptr);
            };
            const uint32_t a = w == 0 ? cut[c] : row_at(k0 + (k1 - k0) * w / T);
            const uint32_t b = w == T - 1 ? cut[c + 1] : row_at(k0 + (k1 - k0) * (w + 1) / T);
            bool ov = false, id = true;
            if (a < b) scan_rows(g, a, b, part[w], cs, slot[c % DEPTH], k0, &ov, &id, check_loss);
            over[(size_t)c * T + w] = ov;
            ident[(size_t)c * T + w] = id;
            done[c].fetch_add(1, std::memory_order_acq_rel);
        }
    }
    // main thread, device ready: upload the pieces as the scan finishes them
    srt_status run(srt_plan *p, srt_err *err) {
        hipStream_t M = p->stream;
        HIP_TRY(hipMalloc(&p->d_up32, (size_t)DEPTH * PE * 4), "hipMalloc(upload slots)");
        for (int i = 0; i < DEPTH; ++i) HIP_TRY(hipEventCreateWithFlags(&ev[i], hipEventDisableTiming), "event");
        for (uint32_t c = 0; c < P; ++c) {
            while (done[c].load(std::memory_order_acquire) < T) std::this_thread::yield();
            bool lat_ok = true, id = true;
            for (int w = 0; w < T; ++w) {
                lat_ok &= !over[(size_t)c * T + w];
                id &= ident[(size_t)c * T + w] != 0;
            }
            const uint64_t k0 = g->row_ptr[cut[c]], cnt = g->row_ptr[cut[c + 1]] - k0;
            uint32_t *dslot = p->d_up32 + (uint64_t)(c % DEPTH) * PE;
            if (cnt && lat_ok) {
                HIP_TRY(hipMemcpyAsync(dslot, slot[c % DEPTH], cnt * 4, hipMemcpyHostToDevice, M), "upload (lat)");
                srt::widen_u32(p->d_lat + k0, dslot, cnt, M);
            } else if (cnt) {
                HIP_TRY(hipMemcpyAsync(p->d_lat + k0, g->lat_ns + k0, cnt * 8, hipMemcpyHostToDevice, M), "upload (lat)");
            }
            HIP_TRY(hipEventRecord(ev[c % DEPTH], M), "event");
            if (cnt && id) srt::iota_rows(p->d_col + k0, cnt, g->n_nodes, M);
            else if (cnt)
                HIP_TRY(hipMemcpyAsync(p->d_col + k0, g->col + k0, cnt * 4, hipMemcpyHostToDevice, M), "upload (col)");
            if (c + DEPTH < P) {
                // the slot of piece c + DEPTH is piece c's: free once its copy is done
                HIP_TRY(hipEventSynchronize(ev[c % DEPTH]), "sync (upload)");
                ready.store((int)(c + DEPTH), std::memory_order_release);
            }
        }
        return SRT_OK;
    }
    // every thread joined, the stats merged, the slots drained, the pool free
    void finish(CsrStats *cs) {
        ready.store((int)P);
        for (auto &th : pool) th.join();
        pool.clear();
        merge_stats(part, g->n_nodes, cs);
        for (int i = 0; i < DEPTH; ++i)
            if (ev[i]) {
                (void)hipEventSynchronize(ev[i]);
                (void)hipEventDestroy(ev[i]);
                ev[i] = nullptr;
            }
        if (lk.owns_lock()) lk.unlock();
    }
    ~PieceUpload() {
        if (on && !pool.empty()) {
            ready.store((int)P);
            for (auto &th : pool) th.join();
        }
    }
};

// End-to-end builds: the edge losses uploaded while the closure runs, through
// the pinned staging in 64 MB pieces (host threads copy a piece into a slot,
// 3 in flight, the DMA runs at the link rate instead of the pageable ~21 GB/s:
// C3's 1 GB 48 ms -> ~25, under the 46 ms closure), then range-checked on the
// device (srt::loss_check; the host scan skipped the losses).  Falls back to
// one pageable copy when the staging is busy.
struct LossUpload {
    static constexpr int DEPTH = 3;
    static constexpr uint64_t PE = 1ull << 24;  // floats a piece
    const float *src = nullptr;
    uint64_t m = 0;
    uint32_t P = 0;
    int T = 1;
    std::unique_ptr<std::atomic<int>[]> done;
    std::atomic<int> ready{-1};
    std::vector<std::thread> pool;
    float *slot[DEPTH] = {};
    hipEvent_t ev[DEPTH] = {};

    void work(int w) {
        for (uint32_t c = 0; c < P; ++c) {
            while (ready.load(std::memory_order_acquire) < (int)c) std::this_thread::yield();
            const uint64_t k0 = (uint64_t)c * PE, cnt = std::min(PE, m - k0);
            const uint64_t a = cnt * w / T, b = cnt * (w + 1) / T;
            std::memcpy(slot[c % DEPTH] + a, src + k0 + a, (b - a) * 4);
            done[c].fetch_add(1, std::memory_order_acq_rel);
        }
    }
    // on stream `up`; the check's result goes to p->d_lossbad
    srt_status run(srt_plan *p, hipStream_t up, srt_err *err) {
        std::unique_lock<std::mutex> lk(g_pinned.m, std::try_to_lock);
        if (!lk.owns_lock() || g_pinned.bytes < DEPTH * PE * 4) {
            HIP_TRY(hipMemcpyAsync(p->d_loss, src, m * 4, hipMemcpyHostToDevice, up), "upload (loss)");
            HIP_TRY(hipMemsetAsync(p->d_lossbad, 0xff, 8, up), "memset (loss check)");
            srt::loss_check(p->d_loss, m, 0, p->d_lossbad, up);
            return SRT_OK;
        }
        for (int i = 0; i < DEPTH; ++i) slot[i] = reinterpret_cast<float *>(g_pinned.buf) + (uint64_t)i * PE;
        P = (uint32_t)((m + PE - 1) / PE);
        T = std::min(16, host_threads(m));
        done.reset(new std::atomic<int>[P]);
        for (uint32_t c = 0; c < P; ++c) done[c].store(0);
        ready.store(std::min<int>(DEPTH, (int)P) - 1);
        for (int w = 1; w < T; ++w) pool.emplace_back([this, w] { work(w); });
        srt_status st = SRT_OK;
        hipError_t e = hipSuccess;
        using clk = std::chrono::steady_clock;
        double w_copy = 0, w_dma = 0;  // SRT_TRACE: waits on the host copies / on the DMA
        const auto t_start = clk::now();
        for (int i = 0; i < DEPTH && e == hipSuccess; ++i) e = hipEventCreateWithFlags(&ev[i], hipEventDisableTiming);
        for (uint32_t c = 0; c < P && e == hipSuccess; ++c) {
            // this thread copies its share too, then queues the piece
            {
                while (ready.load(std::memory_order_acquire) < (int)c) std::this_thread::yield();
                const uint64_t k0 = (uint64_t)c * PE, cnt = std::min(PE, m - k0);
                std::memcpy(slot[c % DEPTH], src + k0, (cnt / T) * 4);
                done[c].fetch_add(1, std::memory_order_acq_rel);
            }
            auto t0 = clk::now();
            while (done[c].load(std::memory_order_acquire) < T) std::this_thread::yield();
            w_copy += std::chrono::duration<double, std::milli>(clk::now() - t0).count();
            const uint64_t k0 = (uint64_t)c * PE, cnt = std::min(PE, m - k0);
            e = hipMemcpyAsync(p->d_loss + k0, slot[c % DEPTH], cnt * 4, hipMemcpyHostToDevice, up);
            if (e == hipSuccess) e = hipEventRecord(ev[c % DEPTH], up);
            if (e == hipSuccess && c + DEPTH < P) {
                t0 = clk::now();
                e = hipEventSynchronize(ev[c % DEPTH]);  // slot c's copy done: piece c + DEPTH may fill it
                w_dma += std::chrono::duration<double, std::milli>(clk::now() - t0).count();
                ready.store((int)(c + DEPTH), std::memory_order_release);
            }
        }
        ready.store((int)P);  // release the workers on any error
        for (auto &th : pool) th.join();
        // one check behind all the copies: a kernel (the memset's fill kernel
        // too) queued before or between them waits for CUs the closure holds,
        // and every later copy with it (measured: the 1 GB took the closure's
        // 48 ms)
        if (e == hipSuccess) e = hipMemsetAsync(p->d_lossbad, 0xff, 8, up);
        if (e == hipSuccess) srt::loss_check(p->d_loss, m, 0, p->d_lossbad, up);
        if (std::getenv("SRT_TRACE"))
            std::fprintf(stderr, "[srt] loss pieces: %u x %llu MB, %d threads, %.1f ms: waited %.1f ms on copies, %.1f on DMA\n",
                         P, (unsigned long long)(PE * 4 >> 20), T,
                         std::chrono::duration<double, std::milli>(clk::now() - t_start).count(), w_copy, w_dma);
        for (int i = 0; i < DEPTH; ++i)
            if (ev[i]) {
                (void)hipEventSynchronize(ev[i]);  // the staging is free for the download
                (void)hipEventDestroy(ev[i]);
            }
        if (e != hipSuccess) st = hip_fail(err, e, "upload (loss pieces)");
        return st;
    }
};

// Choose the closure's key representation and prove it exact.
//
// Keys are path latencies in units of g = gcd of all edge latencies (latency
// only: the loss is recomputed exactly by the loss pass, so no loss bits share
// the key).  Lmax bounds every shortest-path latency: the longest edge for a
// complete graph (a direct edge bounds every pair), else (V-1) * max edge --
// or, tighter, in-eccentricity + out-eccentricity of one node that reaches
// and is reached by every node (fw_ecc_bound: d(u,v) <= d(u,s) + d(s,v)).
// Edges longer than Lmax are then stored saturated at INF (the init kernels).
// Exactness does not depend on the schedule's read order: (1) every stored
// value only decreases from its initial value <= INF, so each operand is <=
// INF and a candidate (sum of two) is <= 2 INF, which the key type holds
// without wrapping (u16 lanes: 0xFFFE; u32: 2^32 - 2) -- no candidate is ever
// corrupted, whatever the grouped / look-ahead / sharded schedules read; (2) a
// candidate below INF is the exact length of a real walk, so no stored value
// drops below the true distance d; (3) the schedule's values are never above
// the sequential Floyd-Warshall's (its candidates are formed from operands at
// least as tight), which ends at d.  So the closure ends at d exactly when
// every finite d < INF -- Lmax < INF.  The test below asks for 2 Lmax + 1 <
// INF, a margin kept from the r01 packed (latency, loss) keys.  Below 2^53 the
// keys may be f64 (v_add_f64 / v_min_f64), below 2^62 u64, and below
// KEY32_INF (2^31 - 1) u32; u16 below KEY16_INF.  Lmax < 2^32 - 1
// additionally lets the loss pass keep latencies as u32.  Knob
// SRT_FW_KEY=u32|f64|u64 (measurement / A-B parity only) skips the narrower
// representations.
bool choose_key_params(const CsrStats &cs, uint32_t V, uint64_t ecc_units, KeyParams *kp, int *key_type, bool *f16,
                       std::string *why) {
    kp->g = cs.gcd;
    const uint64_t maxu = cs.maxlat / cs.gcd;
    unsigned __int128 Lmax = cs.complete ? (unsigned __int128)maxu : (unsigned __int128)(V ? V - 1 : 0) * maxu;
    // the eccentricity bound (fw_ecc_bound), when the sweeps found one
    if (ecc_units != ~0ull && (unsigned __int128)ecc_units < Lmax) Lmax = ecc_units;
    kp->lmax = Lmax > (unsigned __int128)~0ull ? ~0ull : (uint64_t)Lmax;
    kp->lat32 = Lmax < 0xffffffffull;
    // knob SRT_FW_KEY = u16 / u32 / f64 / u64: the narrowest key allowed (A/B, tests)
    const char *force = std::getenv("SRT_FW_KEY");
    const bool allow16 = !force || std::strcmp(force, "u16") == 0;
    const int min_type = !force ? srt::KEY_U32 : std::strcmp(force, "u64") == 0 ? srt::KEY_U64
                         : std::strcmp(force, "f64") == 0 ? srt::KEY_F64 : srt::KEY_U32;
    *f16 = false;
    if (allow16 && 2 * Lmax + 1 < (unsigned __int128)srt::KEY16_INF) {
        *key_type = srt::KEY_U16;
        // f16 integer arithmetic on the same 2-byte keys (0.75 VALU slot per
        // relaxation instead of 1): every finite distance < 1024 = F16 INF,
        // so candidates stay <= 2048, exact in f16 (srt_fw.hip).  SRT_FW_KEY=u16
        // keeps integer arithmetic (A/B parity tests).
        *f16 = !force && Lmax < 1024;
        return true;
    }
    if (min_type <= srt::KEY_U32 && 2 * Lmax + 1 < (unsigned __int128)srt::KEY32_INF) {
        *key_type = srt::KEY_U32;
        return true;
    }
    if (min_type <= srt::KEY_F64 && 2 * Lmax + 1 < ((unsigned __int128)1 << 53)) {
        *key_type = srt::KEY_F64;
        return true;
    }
    if (2 * Lmax + 1 < ((unsigned __int128)1 << 62)) {
        *key_type = srt::KEY_U64;
        return true;
    }
    *why = "the latency range does not fit a 62-bit exact key";
    return false;
}

// Teardown of the one-call builds' plans behind their return (C3: ~6 ms of
// stream syncs and hipFree of ~5 GB): one worker thread, plans queued; an
// allocation that fails drains the queue and retries; joined at exit.
struct Reaper {
    std::mutex m;
    std::condition_variable cv, idle;
    std::deque<srt_plan *> q;
    std::thread th;
    bool busy = false, stop = false;
};
Reaper g_reap;

void reap_worker() {
    std::unique_lock<std::mutex> lk(g_reap.m);
    for (;;) {
        g_reap.cv.wait(lk, [] { return g_reap.stop || !g_reap.q.empty(); });
        if (g_reap.q.empty()) return;  // stopping, nothing left
        srt_plan *p = g_reap.q.front();
        g_reap.q.pop_front();
        g_reap.busy = true;
        lk.unlock();
        srt_plan_destroy(p);
        lk.lock();
        g_reap.busy = false;
        if (g_reap.q.empty()) g_reap.idle.notify_all();
    }
}

// every queued plan destroyed
void reap_drain() {
    std::unique_lock<std::mutex> lk(g_reap.m);
    g_reap.idle.wait(lk, [] { return g_reap.q.empty() && !g_reap.busy; });
}

// registered after the HIP runtime started, so it runs before its teardown
void reap_stop_at_exit() {
    {
        std::lock_guard<std::mutex> lk(g_reap.m);
        g_reap.stop = true;
    }
    g_reap.cv.notify_all();
    if (g_reap.th.joinable()) g_reap.th.join();
}

void reap_async(srt_plan *p) {
    static std::once_flag once;
    std::call_once(once, [] {
        g_reap.th = std::thread(reap_worker);
        std::atexit(reap_stop_at_exit);
    });
    {
        std::lock_guard<std::mutex> lk(g_reap.m);
        g_reap.q.push_back(p);
    }
    g_reap.cv.notify_one();
}

// Streams and events of destroyed plans, kept for the next plan on the same
// device: creating a plan's 3 streams, 6 events and the ~2 per 128-pivot
// round timing events of the closure cost ~4-6 ms (C3).  At most 4 sets.
struct StreamSet {
    int device = -1;
    hipStream_t stream = nullptr, side = nullptr, comm = nullptr;
    hipEvent_t begin = nullptr, end = nullptr, cross = nullptr, pivot = nullptr, row = nullptr, bcast = nullptr;
    std::vector<hipEvent_t> ev, ev_tail;
};
struct StreamPool {
    std::mutex m;
    std::vector<StreamSet> sets;
};
StreamPool g_streams;

bool take_stream_set(int device, srt_plan *p) {
    std::lock_guard<std::mutex> lk(g_streams.m);
    for (size_t i = 0; i < g_streams.sets.size(); ++i)
        if (g_streams.sets[i].device == device) {
            StreamSet &x = g_streams.sets[i];
            p->stream = x.stream;
            p->side_stream = x.side;
            p->comm_stream = x.comm;
            p->ev_begin = x.begin;
            p->ev_end = x.end;
            p->ev_cross = x.cross;
            p->ev_pivot = x.pivot;
            p->ev_row = x.row;
            p->ev_bcast = x.bcast;
            p->ev.swap(x.ev);
            p->ev_tail.swap(x.ev_tail);
            g_streams.sets.erase(g_streams.sets.begin() + i);
            return true;
        }
    return false;
}

// the plan's (synchronised) streams and events into the pool; false: full
bool give_stream_set(srt_plan *p) {
    if (!p->own_stream || !p->stream || !p->side_stream || !p->comm_stream || !p->ev_begin || !p->ev_end ||
        !p->ev_cross || !p->ev_pivot || !p->ev_row || !p->ev_bcast)
        return false;
    std::lock_guard<std::mutex> lk(g_streams.m);
    if (g_streams.sets.size() >= 4) return false;
    StreamSet x;
    x.device = p->device;
    x.stream = p->stream;
    x.side = p->side_stream;
    x.comm = p->comm_stream;
    x.begin = p->ev_begin;
    x.end = p->ev_end;
    x.cross = p->ev_cross;
    x.pivot = p->ev_pivot;
    x.row = p->ev_row;
    x.bcast = p->ev_bcast;
    x.ev.swap(p->ev);
    x.ev_tail.swap(p->ev_tail);
    g_streams.sets.push_back(std::move(x));
    p->stream = p->side_stream = p->comm_stream = nullptr;
    p->ev_begin = p->ev_end = p->ev_cross = p->ev_pivot = p->ev_row = p->ev_bcast = nullptr;
    return true;
}

template <typename T>
srt_status dmalloc(T **p, size_t count, srt_err *err) {
    void *ptr = nullptr;
    hipError_t e = hipMalloc(&ptr, std::max<size_t>(count, 1) * sizeof(T));
    if (e == hipErrorOutOfMemory) {  // plans still being torn down: wait for them once
        (void)hipGetLastError();
        reap_drain();
        e = hipMalloc(&ptr, std::max<size_t>(count, 1) * sizeof(T));
    }
    if (e != hipSuccess) return hip_fail(err, e, "hipMalloc");
    *p = (T *)ptr;
    return SRT_OK;
}

void free_plan_buffers(srt_plan *p) {
    if (p->loss_checker.joinable()) p->loss_checker.join();  // it writes h_lossbad
    hipFree(p->d_lidx);
    hipFree(p->d_row_ptr);
    hipFree(p->d_col);
    hipFree(p->d_lat);
    hipFree(p->d_lat16);
    hipFree(p->d_rowctr);
    hipFree(p->d_loss);
    hipFree(p->d_nodes);
    hipFree(p->d_D);
    hipFree(p->d_out_lat);
    hipFree(p->d_out_loss);
    hipFree(p->d_sl_lat);
    hipFree(p->d_sl_loss);
    hipFree(p->d_stats);
    hipFree(p->d_pack);
    hipFree(p->d_pack8);
    hipFree(p->d_up32);
    hipFree(p->d_flag32);
    hipFree(p->d_tl_all);
    hipFree(p->d_tl_cnt);
    hipFree(p->d_tl_cross);
    hipFree(p->d_rowslots);
    hipFree(p->d_fbuf);
    hipFree(p->d_draws);
    hipFree(p->d_pkt_tab);
    hipFree(p->d_lvl_offstage);
    hipFree(p->d_lvl_counts);
    hipFree(p->d_pkt_bad);
    hipFree(p->d_in_ptr);
    hipFree(p->d_sperm);
    hipFree(p->d_in_edge);
    hipFree(p->d_sD);
    hipFree(p->d_spend);
    hipFree(p->d_smask);
    hipFree(p->d_sflag);
    hipFree(p->d_sact);
    hipFree(p->d_fl);
    hipFree(p->d_fp);
    hipFree(p->d_ftight);
    hipFree(p->d_fce);
    hipFree(p->d_fcnt);
    hipFree(p->d_fctl);
    hipFree(p->d_fchg);
    hipFree(p->d_fact);
    hipFree(p->d_fdone);
    hipFree(p->d_fsb);
    hipFree(p->d_ffin);
    hipFree(p->d_fnodes);
    hipFree(p->d_frow_ptr);
    hipFree(p->d_fcol);
    hipFree(p->d_fimp);
    if (p->h_fimp) hipHostFree(p->h_fimp);
    if (p->d_lossbad) hipFree(p->d_lossbad);
    if (p->h_lossbad) hipHostFree(p->h_lossbad);
    hipFree(p->d_rstats);
    hipFree(p->d_lvisit);
    hipFree(p->d_lmem);
    hipFree(p->d_ev_scratch);
    hipFree(p->d_tflag);
    hipFree(p->d_tcnt);
    hipFree(p->d_tptr);
    hipFree(p->d_tu);
    hipFree(p->d_tw);
    hipFree(p->d_teb);
    hipFree(p->d_tpk);
    hipFree(p->d_tpk2);
    hipFree(p->d_tsort_tmp);
    hipFree(p->d_tcls);
    hipFree(p->d_tcw);
    hipFree(p->d_ev_bad);
    hipFree(p->d_tccnt);
    hipFree(p->d_tscan_tmp);
    hipFree(p->d_tmaxw);
    hipFree(p->d_lscratch);
    hipFree(p->d_lrows);
    hipFree(p->d_slat);
    hipFree(p->d_sloss);
    hipFree(p->d_tlist);
    hipFree(p->d_tinfo);
    hipFree(p->d_tcursor);
    if (p->h_tinfo) hipHostFree(p->h_tinfo);
    if (p->h_sflag) hipHostFree(p->h_sflag);
    if (p->h_tcount) hipHostFree(p->h_tcount);
}

// Sparse SSSP key (srt_sssp.hip): latency in units of g in the high 32 bits.
// A stored value is a simple path (<= V-1 edges) and a candidate adds one
// edge, so V * max_edge_latency / g < 2^32 - 1 keeps every sum exact and
// below the all-ones "unreached" key.
bool sssp_params(const CsrStats &cs, uint32_t V, std::string *why) {
    if ((unsigned __int128)V * (cs.maxlat / cs.gcd) >= 0xffffffffull) {
        *why = "V * max edge latency exceeds the 32-bit latency field of the SSSP key";
        return false;
    }
    return true;
}

// Family prices for AUTO, seconds on one MI355X, from the measured rates of
// DESIGN.md 4 (rest launches by key type, r03 profiles; sparse builds r04).
// Dense: Vp^3 relaxations (half on the triangle schedule: 2-byte keys on a
// symmetric graph), at least ~80 us a 128-pivot round (the chain: C2 4k), plus
// the exact-loss fold (C3: 7.0 ms for 16k x 16k pairs).  Sparse: one unit per
// (source, in-edge or vertex) visited, at the C4 rate of the frontier sweeps
// (u16 latencies) or of the packed-key sweeps, at least ~1 ms a launch of
// sources (its ~60 dependent sweeps).
double price_fw(uint32_t Vp, uint32_t n, uint32_t V, int key_type, bool f16, bool sym) {
    const double rate = f16                          ? 4.3e13   // C3 rest: 1.45 ms / 6.26e10
                        : key_type == srt::KEY_U16 ? 3.3e13     // 1.90 ms (r02)
                        : key_type == srt::KEY_U32 ? 1.25e13    // 4.82-5.19 ms
                        : key_type == srt::KEY_F64 ? 8e12       // ~half the u32 mix, not profiled
                                                   : 4e12;      // u64: ~1/3 of u32's mix, not profiled
    const bool tri = sym && (f16 || key_type == srt::KEY_U16);
    const double relax = (double)Vp * Vp * Vp * (tri ? 0.5 : 1.0);
    return std::max(relax / rate, (double)(Vp / 128) * 80e-6) + (double)n * V * 2.6e-11;
}
// Level solve: a row walks the probe row's edge count plus ~4 passes over
// the row's V levels (init, the level collections), at the level fold's
// measured cost per visit (C3: 4.56 ms for 16k rows of ~160k visits), and
// writes its 12-byte table row.
double price_level(uint32_t n, uint32_t V, uint64_t visits) {
    return (double)n * ((double)visits + 4.0 * V) * 1.8e-12 + (double)n * n * 12.0 / 5e12 + 3e-4;
}
double price_sparse(uint32_t n, uint64_t n_in, uint32_t V, bool frontier) {
    const double units = (double)n * ((double)n_in + V);
    const double per = frontier ? 1.19e-11 : 1.73e-11;  // C4: 9e10 units in 1.07 s / 1.56 s
    const double launches = std::ceil((double)n / (frontier ? 8192.0 : 4096.0));
    return std::max(units * per, launches * 1e-3);
}

// Pull-form adjacency for the sweep: for every v, the entries u -> v of every
// row u (petgraph edges(u): directed outgoing / undirected incident), minus
// self-loops (they never shorten a path; the diagonal is the raw self-loop).
void build_in_edges(const srt_csr *g, uint64_t gunit, uint64_t n_in, std::vector<uint64_t> *ptr,
                    std::vector<srt::InEdge> *edges) {
    const uint32_t V = g->n_nodes;
    ptr->assign((size_t)V + 1, 0);
    for (uint32_t u = 0; u < V; ++u)
        for (uint64_t k = g->row_ptr[u]; k < g->row_ptr[u + 1]; ++k)
            if (g->col[k] != u) (*ptr)[g->col[k] + 1]++;
    for (uint32_t v = 0; v < V; ++v) (*ptr)[v + 1] += (*ptr)[v];
    edges->resize(std::max<uint64_t>(n_in, 1));
    std::vector<uint64_t> fill(ptr->begin(), ptr->end() - 1);
    for (uint32_t u = 0; u < V; ++u)
        for (uint64_t k = g->row_ptr[u]; k < g->row_ptr[u + 1]; ++k) {
            const uint32_t v = g->col[k];
            if (v == u) continue;
            srt::InEdge e;
            e.u = u;
            e.w = (uint32_t)(g->lat_ns[k] / gunit);
            e.eb = 1.0f - g->loss[k];
            e.pad = 0;
            (*edges)[fill[v]++] = e;
        }
}

// Is the latency adjacency symmetric (every u -> v of latency w has a v -> u of
// latency w, as multisets -- petgraph undirected graphs are)?  Then every
// shortest latency is symmetric, L(s, v) = L(v, s), which the frontier sweeps
// use to seed a launch from the rows of the earlier ones.  Per vertex: the
// in-edges (u, w) against the out-row (col, lat / g), both sorted; host threads
// over vertex ranges.
bool latency_symmetric(const srt_csr *g, const std::vector<uint64_t> &in_ptr, const std::vector<srt::InEdge> &in_edge,
                       uint64_t gunit) {
    const uint32_t V = g->n_nodes;
    const unsigned nt = std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
    std::vector<uint8_t> bad(nt, 0);
    std::vector<std::thread> th;
    for (unsigned t = 0; t < nt; ++t)
        th.emplace_back([&, t] {
            std::vector<uint64_t> a, b;
            for (uint32_t v = (uint32_t)((uint64_t)V * t / nt); v < (uint32_t)((uint64_t)V * (t + 1) / nt) && !bad[t];
                 ++v) {
                a.clear();
                b.clear();
                for (uint64_t k = in_ptr[v]; k < in_ptr[v + 1]; ++k)
                    a.push_back((uint64_t)in_edge[k].u << 32 | in_edge[k].w);
                for (uint64_t k = g->row_ptr[v]; k < g->row_ptr[v + 1]; ++k)
                    if (g->col[k] != v) b.push_back((uint64_t)g->col[k] << 32 | (uint32_t)(g->lat_ns[k] / gunit));
                if (a.size() != b.size()) {
                    bad[t] = 1;
                    break;
                }
                std::sort(a.begin(), a.end());
                std::sort(b.begin(), b.end());
                if (a != b) bad[t] = 1;
            }
        });
    for (auto &x : th) x.join();
    for (uint8_t x : bad)
        if (x) return false;
    return true;
}

// Source order of the sparse sweeps: the level order of a shortest-latency
// tree from the highest-degree vertex (then from the lowest-numbered vertex
// not yet reached): the root, its tree children, theirs, ... each parent's
// children together.  The sweeps put table rows in this order into their
// words, lanes (8 sources) and 128-B lines (32 sources); sources at the same
// tree depth under nearby parents reach most targets along paths of the same
// hop count, so a word's labels change at the same vertices in the same
// sweeps.  C4's graph (tools measurement on the host, hop counts of the
// shortest-path trees of 32-source lines over all targets): 3.1 distinct hop
// counts a line in this order, 9.7 in plain breadth-first order from the same
// root, 7.5 in tree depth-first order.  Measured on C4: loss sweeps 266 -> 214
// ms a build; but as the order of the launches (which sources come first) it
// costs the symmetric seeding (latency sweeps 94 -> 142 ms), so the frontier
// composes launches in breadth-first order (hop_rank) and orders rows within a
// launch by this rank.
// plain breadth-first discovery order from the same root (knob SRT_SSSP_ORDER=2, A/B)
std::vector<uint32_t> hop_rank(const srt_csr *g) {
    const uint32_t V = g->n_nodes;
    std::vector<uint32_t> rank(V, ~0u), q;
    q.reserve(V);
    uint32_t start = 0;
    uint64_t best = 0;
    for (uint32_t u = 0; u < V; ++u)
        if (g->row_ptr[u + 1] - g->row_ptr[u] > best) best = g->row_ptr[u + 1] - g->row_ptr[u], start = u;
    uint32_t next = 0;
    for (uint32_t root = start, scan = 0; next < V;) {
        if (rank[root] == ~0u) {
            rank[root] = next++;
            q.push_back(root);
            for (size_t h = q.size() - 1; h < q.size(); ++h)
                for (uint64_t k = g->row_ptr[q[h]]; k < g->row_ptr[q[h] + 1]; ++k) {
                    const uint32_t v = g->col[k];
                    if (v < V && rank[v] == ~0u) {
                        rank[v] = next++;
                        q.push_back(v);
                    }
                }
        }
        while (scan < V && rank[scan] != ~0u) ++scan;
        root = scan;
    }
    return rank;
}

std::vector<uint32_t> spt_rank(const srt_csr *g) {
    const uint32_t V = g->n_nodes, NONE = ~0u;
    std::vector<uint32_t> rank(V, NONE), first(V, NONE), last(V, NONE), sib(V, NONE), q;
    std::vector<uint64_t> dist(V, ~0ull);
    std::vector<uint32_t> pred(V, NONE);
    std::vector<uint8_t> done(V, 0);
    q.reserve(V);
    uint32_t start = 0;
    uint64_t best = 0;
    for (uint32_t u = 0; u < V; ++u)
        if (g->row_ptr[u + 1] - g->row_ptr[u] > best) best = g->row_ptr[u + 1] - g->row_ptr[u], start = u;
    typedef std::pair<uint64_t, uint32_t> Item;
    std::priority_queue<Item, std::vector<Item>, std::greater<Item>> heap;
    uint32_t next = 0;
    for (uint32_t root = start, scan = 0; next < V;) {
        if (rank[root] == NONE) {
            // Dijkstra over the adjacency's latencies; a vertex joins its
            // parent's child list when settled (children in settle order)
            dist[root] = 0;
            heap.push({0, root});
            while (!heap.empty()) {
                const Item it = heap.top();
                heap.pop();
                const uint32_t u = it.second;
                if (done[u] || it.first != dist[u]) continue;
                done[u] = 1;
                if (u != root) {
                    const uint32_t pu = pred[u];
                    if (last[pu] == NONE) first[pu] = u;
                    else sib[last[pu]] = u;
                    last[pu] = u;
                }
                for (uint64_t k = g->row_ptr[u]; k < g->row_ptr[u + 1]; ++k) {
                    const uint32_t v = g->col[k];
                    if (v >= V || done[v]) continue;
                    const uint64_t d = it.first + g->lat_ns[k];
                    if (d < dist[v]) {
                        dist[v] = d;
                        pred[v] = u;
                        heap.push({d, v});
                    }
                }
            }
            // the tree's level order
            q.clear();
            q.push_back(root);
            rank[root] = next++;
            for (size_t h = 0; h < q.size(); ++h)
                for (uint32_t c = first[q[h]]; c != NONE; c = sib[c]) {
                    rank[c] = next++;
                    q.push_back(c);
                }
        }
        while (scan < V && rank[scan] != NONE) ++scan;
        root = scan;
    }
    return rank;
}

}  // namespace

extern "C" {

int srt_abi_version(void) { return SRT_ABI_VERSION; }

int srt_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}

namespace {
srt_status plan_create_impl(const srt_csr *g, const uint32_t *nodes, uint32_t n, const srt_opts *opts,
                            srt_plan **plan_out, srt_err *err, bool defer_loss);
}

srt_status srt_plan_create(const srt_csr *g, const uint32_t *nodes, uint32_t n,
                           const srt_opts *opts, srt_plan **plan_out, srt_err *err) {
    return plan_create_impl(g, nodes, n, opts, plan_out, err, false);
}

namespace {
// defer_loss (end-to-end build only): the edge-loss array is uploaded by
// run_tail, while the closure runs -- g->loss must stay valid until then
srt_status plan_create_impl(const srt_csr *g, const uint32_t *nodes, uint32_t n, const srt_opts *opts,
                            srt_plan **plan_out, srt_err *err, bool defer_loss) {
    clear_err(err);
    srt::init_wait();  // a pending srt_init_async finishes before any device work
    // plans an earlier one-call build queued for teardown free their HBM
    // before this plan sizes itself (hipMemGetInfo) or allocates anything
    reap_drain();
    Trace tr;
    if (!g || !plan_out || (n && !nodes) || !g->row_ptr || (g->n_adj && (!g->col || !g->lat_ns || !g->loss))) {
        set_err(err, SRT_ERR_INVALID, "null argument");
        return SRT_ERR_INVALID;
    }
    *plan_out = nullptr;
    // in-use nodes must be valid and unique (they come from a HashSet)
    std::vector<uint8_t> seen(g->n_nodes, 0);
    for (uint32_t i = 0; i < n; ++i) {
        if (nodes[i] >= g->n_nodes || seen[nodes[i]]) {
            set_err(err, SRT_ERR_INVALID, "in-use node list has an out-of-range or duplicate NodeIndex");
            return SRT_ERR_INVALID;
        }
        seen[nodes[i]] = 1;
    }
    if (g->row_ptr[g->n_nodes] != g->n_adj) {
        set_err(err, SRT_ERR_INVALID, "row_ptr[n_nodes] != n_adj");
        return SRT_ERR_INVALID;
    }
    srt_plan *p = new (std::nothrow) srt_plan();
    if (!p) {
        set_err(err, SRT_ERR_OOM, "out of host memory");
        return SRT_ERR_OOM;
    }
    p->V = g->n_nodes;
    p->Vp = ((g->n_nodes + srt::FW_B - 1) / srt::FW_B) * srt::FW_B;
    if (p->Vp == 0) p->Vp = srt::FW_B;
    p->rb0 = 0;
    p->rb1 = p->Vp / srt::FW_B;
    p->n = n;
    p->n_adj = g->n_adj;
    p->nodes.assign(nodes, nodes + n);
    p->identity_nodes = (n == g->n_nodes);
    for (uint32_t i = 0; i < n && p->identity_nodes; ++i) p->identity_nodes = nodes[i] == i;
    if (g->node_ids) p->node_ids.assign(g->node_ids, g->node_ids + g->n_nodes);

    // 1. the CSR scan (validation + statistics) on host threads while this
    //    thread sets up the device and uploads the CSR
    CsrStats cs;
    PieceUpload pu;
    const bool piped = pu.init(g, &cs, !defer_loss);
    std::thread scanner;
    if (!piped) scanner = std::thread([&] { csr_scan(g, &cs, !defer_loss); });
    srt_err derr{};
    const srt_status dst = [&]() -> srt_status {
        srt_err *err = &derr;
        int dev = opts && opts->device >= 0 ? opts->device : -1;
        if (dev < 0 && hipGetDevice(&dev) != hipSuccess) dev = 0;
        p->device = dev;
        hipError_t e = hipSetDevice(dev);
        if (e != hipSuccess) return hip_fail(err, e, "hipSetDevice");
        p->own_stream = true;
        if (!take_stream_set(dev, p)) {
            e = hipStreamCreateWithFlags(&p->stream, hipStreamNonBlocking);
            if (e != hipSuccess) return hip_fail(err, e, "hipStreamCreate");
            int lo = 0, hi = 0;
            (void)hipDeviceGetStreamPriorityRange(&lo, &hi);
            e = hipStreamCreateWithPriority(&p->side_stream, hipStreamNonBlocking, hi);
            if (e == hipSuccess) e = hipStreamCreateWithPriority(&p->comm_stream, hipStreamNonBlocking, hi);
            if (e != hipSuccess) return hip_fail(err, e, "hipStreamCreateWithPriority");
            (void)hipEventCreate(&p->ev_begin);
            (void)hipEventCreate(&p->ev_end);
            // the stream-to-stream events of the look-ahead schedule (the
            // system-scope fence is kept: skipping it measured no faster)
            const unsigned sync_fl = hipEventDisableTiming;
            (void)hipEventCreateWithFlags(&p->ev_cross, sync_fl);
            (void)hipEventCreateWithFlags(&p->ev_pivot, sync_fl);
            (void)hipEventCreateWithFlags(&p->ev_row, sync_fl);
            (void)hipEventCreateWithFlags(&p->ev_bcast, sync_fl);
        }
        tr.mark("create: streams + events");
        srt_status st;
        if ((st = dmalloc(&p->d_row_ptr, (size_t)g->n_nodes + 1, err)) != SRT_OK ||
            (st = dmalloc(&p->d_col, g->n_adj, err)) != SRT_OK || (st = dmalloc(&p->d_lat, g->n_adj, err)) != SRT_OK ||
            (st = dmalloc(&p->d_loss, g->n_adj, err)) != SRT_OK || (st = dmalloc(&p->d_nodes, n, err)) != SRT_OK ||
            (st = dmalloc(&p->d_sl_lat, n, err)) != SRT_OK || (st = dmalloc(&p->d_sl_loss, n, err)) != SRT_OK ||
            (st = dmalloc(&p->d_stats, 2, err)) != SRT_OK || (st = dmalloc(&p->d_rstats, 2, err)) != SRT_OK)
            return st;
        tr.mark("create: CSR device buffers");
        auto up = [&](void *dst, const void *src, size_t bytes) -> hipError_t {
            if (!bytes) return hipSuccess;
            return hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, p->stream);
        };
        if (defer_loss) p->h_loss_defer = g->loss;
        if ((e = up(p->d_row_ptr, g->row_ptr, ((size_t)g->n_nodes + 1) * 8)) != hipSuccess ||
            (e = up(p->d_nodes, nodes, (size_t)n * 4)) != hipSuccess ||
            (e = piped ? hipSuccess : up(p->d_col, g->col, g->n_adj * 4)) != hipSuccess ||
            (e = piped ? hipSuccess : up(p->d_lat, g->lat_ns, g->n_adj * 8)) != hipSuccess)
            return hip_fail(err, e, "upload");
        if (piped && (st = pu.run(p, err)) != SRT_OK) return st;
        if ((e = defer_loss ? hipSuccess : up(p->d_loss, g->loss, g->n_adj * 4)) != hipSuccess)
            return hip_fail(err, e, "upload");
        return SRT_OK;
    }();
    tr.mark(piped ? "create: device setup+piece upload" : "create: device setup+upload");
    if (piped) pu.finish(&cs);
    else scanner.join();
    p->ident_rows = cs.ident;
    {
        bool idn = n == g->n_nodes;
        for (uint32_t j = 0; idn && j < n; ++j) idn = nodes[j] == j;
        p->ident_nodes = idn;
    }
    tr.mark("create: CSR scan (joined)");

    // 2. the reference's errors, in its order: edge attributes (parse time),
    //    then the self-loop of every in-use node in node order (mod.rs:210-217)
    auto fail = [&](srt_status s, const char *msg) {
        srt_plan_destroy(p);
        set_err(err, s, msg);
        return s;
    };
    if (cs.badcol_k != ~0ull) return fail(SRT_ERR_INVALID, "adjacency entry names a node out of range");
    if (cs.zero_k != ~0ull) return fail(SRT_ERR_INVALID, "Edge 'latency' must not be 0");
    if (cs.badloss_k != ~0ull) return fail(SRT_ERR_INVALID, "Edge 'packet_loss' is not in the range [0,1]");
    std::vector<uint64_t> sl_lat(n);
    std::vector<float> sl_loss(n);
    for (uint32_t i = 0; i < n; ++i) {
        const uint32_t u = nodes[i], c = cs.sl_cnt[u];
        if (c != 1) {
            // the losses were left to the device: the parse-time error first
            if (defer_loss && srt::first_bad_loss(g) != ~0ull)
                return fail(SRT_ERR_INVALID, "Edge 'packet_loss' is not in the range [0,1]");
            srt_plan_destroy(p);
            return edge_error(err, (int)c, node_id(g, u), node_id(g, u));
        }
        sl_lat[i] = g->lat_ns[cs.sl_first[u]];
        sl_loss[i] = g->loss[cs.sl_first[u]];
    }
    if (dst != SRT_OK) {
        srt_plan_destroy(p);
        if (err) *err = derr;
        return dst;
    }

    // the kernels of creation (bound proofs, probes, symmetry check) are
    // timed from here on (srt::cspan_*): srt_timing.create_device_ms.  The
    // code objects are loaded first (once per device and process; srt_init
    // does it ahead of time), so a span holds no lazy load of a kernel.
    {
        static std::mutex mu;
        static std::vector<int> loaded;
        std::lock_guard<std::mutex> lk(mu);
        if (std::find(loaded.begin(), loaded.end(), p->device) == loaded.end()) {
            (void)hipSetDevice(p->device);
            if (srt::preload_kernels() == hipSuccess) loaded.push_back(p->device);
        }
    }
    p->in_create = true;
    auto dev_timed = [&](auto &&fn) -> srt_status { return fn(); };

    // 2b. the key-width proof from the real diameter, where the family is
    //     likely dense, the graph is not complete (complete graphs have the
    //     longest-edge bound) and (V-1) * max edge would not allow f16 keys
    uint64_t ecc_units = ~0ull;
    uint32_t ecc_sweeps = 0;
    {
        const uint64_t maxu = cs.maxlat / cs.gcd;
        const uint64_t nin = g->n_adj - cs.selfloops;
        const uint32_t want0 = opts ? opts->algo : (uint32_t)SRT_ALGO_AUTO;
        // priced as if the proof gave 2-byte keys (it decides whether to run it)
        const bool sym = cs.sym_a == cs.sym_b;
        const bool dense_likely = want0 == SRT_ALGO_FW ||
                                  (want0 == SRT_ALGO_AUTO && price_fw(p->Vp, n, p->V, srt::KEY_U16, true, sym) <
                                                                 price_sparse(n, nin, p->V, true));
        // sparse plans need it too: the frontier sweeps keep u16 latencies
        // when every finite distance is below 0xFFFF units (srt_frontier.hip)
        const bool sparse_u16 = !dense_likely && (unsigned __int128)(p->V ? p->V - 1 : 0) * maxu >= 0xffff;
        if (!cs.complete && (dense_likely || sparse_u16) &&
            (unsigned __int128)(p->V ? p->V - 1 : 0) * maxu >= 1024 && !std::getenv("SRT_FW_NO_ECC")) {
            uint64_t b = ~0ull;
            srt_err e2{};
            if (dev_timed([&] { return srt::fw_ecc_bound(p, 512, &b, &ecc_sweeps, &e2); }) != SRT_OK) {
                srt_plan_destroy(p);
                if (err) *err = e2;
                return SRT_ERR_HIP;
            }
            if (b != ~0ull) ecc_units = b / cs.gcd;
        }
    }
    (void)ecc_sweeps;
    tr.mark("create: eccentricity sweeps");

    // 3. kernel family: AUTO takes the cheaper representable one at the
    //    measured rates (price_fw, price_sparse)
    std::string why_fw, why_sssp;
    bool f16 = false;
    const bool fw_ok = choose_key_params(cs, p->V, ecc_units, &p->kp, &p->key_type, &f16, &why_fw);
    // no parallel edges: the FW init can store edge keys instead of atomic-min'ing them
    p->fw_unique_edges = cs.unique;
    const uint64_t n_in = g->n_adj - cs.selfloops;
    const bool sssp_ok = sssp_params(cs, p->V, &why_sssp);
    p->sssp_g = cs.gcd;
    const uint32_t want = opts ? opts->algo : (uint32_t)SRT_ALGO_AUTO;
    if (want > SRT_ALGO_LEVEL) return fail(SRT_ERR_INVALID, "unknown srt_opts.algo");
    // 3a. the level solve (srt_loss.hip level_solve_kernel): asked for, or
    //     AUTO on a graph whose row fits LDS.  The probe proves B, a bound
    //     on every in-use shortest path over the edges <= min(31, max edge)
    //     units; the solve applies when one was found (B <= 31).
    uint64_t lvl_bound = ~0ull, lvl_visits = 0;
    std::string why_lvl =
        "the level solve needs V <= 18400 and every shortest path <= 63 latency units (or 63 buckets as wide "
        "as the shortest edge)";
    {
        const uint64_t maxu = cs.maxlat / cs.gcd;
        const bool fits = p->V >= 2 && p->V <= srt::LEVEL_V_MAX && n >= 1;
        const char *kl = std::getenv("SRT_LEVEL");  // knob: 0 keeps AUTO off the level solve (A/B, tests)
        const bool try_lvl = fits && maxu >= 1 &&
                             (want == SRT_ALGO_LEVEL || (want == SRT_ALGO_AUTO && !(kl && std::atoi(kl) == 0)));
        if (try_lvl) {
            p->kp.g = cs.gcd;
            p->lvl_q = 0;
            p->lvl_maxu = maxu;
            srt_err e2{};
            auto probe_fail = [&]() {
                srt_plan_destroy(p);
                if (err) *err = e2;
                return e2.code ? (srt_status)e2.code : SRT_ERR_HIP;
            };
            // complete graphs in identity rows whose pairs mirror exactly (the
            // latencies here, over every pair; the losses too when they are on
            // the device, else the one-call build checks the losses it
            // gathers): one class CSR, the in-rows being the out-rows
            const char *ks = std::getenv("SRT_LVL_SYM");  // knob: 0 = always build the in-rows (A/B, tests)
            if (cs.complete && !(ks && std::atoi(ks) == 0)) {
                bool sym = false;
                if (dev_timed([&] { return srt::level_sym_check(p, maxu, !defer_loss, &sym, &e2); }) != SRT_OK)
                    return probe_fail();
                p->lvl_sym_lat = p->lvl_sym = sym;
            }
            // levels of one unit
            auto probe = [&](uint64_t wmax, uint32_t wc) {
                return dev_timed([&] { return srt::level_probe(p, wmax, wc, &lvl_bound, &lvl_visits, &e2); });
            };
            // 15 classes first (r06: C1-C3 prove B <= 14 there, and the probe CSR
            // of the edges <= 15 units is half the one at 31), then 31, then 63
            // (each also admits longer paths of short edges: bounds up to wc)
            if (probe(std::min<uint64_t>(15, maxu), 15) != SRT_OK) return probe_fail();
            if (lvl_bound == ~0ull && probe(std::min<uint64_t>(31, maxu), 31) != SRT_OK) return probe_fail();
            if (lvl_bound == ~0ull && probe(std::min<uint64_t>(63, maxu), 63) != SRT_OK) return probe_fail();
            // no bound within 63 units: the quantized solve, buckets of q <= the
            // shortest edge (C3ns: g = 1 ns, edges >= 1 ms), when the shortest
            // paths stay under 64 such buckets
            const char *kq = std::getenv("SRT_LEVEL_Q");  // knob: 0 = integer levels only (A/B, tests)
            if (lvl_bound == ~0ull && !(kq && std::atoi(kq) == 0)) {
                uint64_t mn_ns = ~0ull;
                if (dev_timed([&] { return srt::level_min_edge(p, &mn_ns, &e2); }) != SRT_OK) return probe_fail();
                const uint64_t mu = mn_ns == ~0ull ? 0 : mn_ns / cs.gcd;
                const uint32_t vb = srt::level_vbits(p->V);
                // an entry keeps the remainder w - c q (< q) in 34 - vb bits;
                // latencies up to 64 q stay below 2^31
                const uint64_t q = std::min<uint64_t>(std::min<uint64_t>(mu, 1ull << (34 - vb)), 1ull << 25);
                if (q >= 2) {
                    uint32_t rb = 0;
                    while ((1ull << rb) < q) ++rb;
                    p->lvl_q = (uint32_t)q;
                    p->lvl_rb = rb;
                    p->lvl_vb = vb;
                    if (probe(std::min<uint64_t>(maxu, 32 * q - 1), 31) != SRT_OK) return probe_fail();
                    if (lvl_bound == ~0ull && probe(std::min<uint64_t>(maxu, 64 * q - 1), 63) != SRT_OK)
                        return probe_fail();
                    if (lvl_bound == ~0ull) p->lvl_q = 0;
                }
            }
            // the probe's lists were sized for it; the run builds its own
            p->t_edges = 0;
        }
    }
    const bool lvl_ok = lvl_bound != ~0ull;
    tr.mark("create: level probe");
    int algo = -1;
    std::string auto_note;
    if (want == SRT_ALGO_FW) {
        if (fw_ok) algo = SRT_ALGO_FW;
    } else if (want == SRT_ALGO_SSSP) {
        if (sssp_ok) algo = SRT_ALGO_SSSP;
    } else if (want == SRT_ALGO_LEVEL) {
        if (lvl_ok) algo = SRT_ALGO_LEVEL;
    } else {
        const uint64_t maxu = cs.maxlat / cs.gcd;
        const unsigned __int128 lb = ecc_units != ~0ull ? (unsigned __int128)ecc_units
                                                        : (unsigned __int128)(p->V ? p->V - 1 : 0) * maxu;
        const double t_fw = fw_ok ? price_fw(p->Vp, n, p->V, p->key_type, f16, cs.sym_a == cs.sym_b) : 1e300;
        const double t_sssp = sssp_ok ? price_sparse(n, n_in, p->V, lb < 0xffff) : 1e300;
        const double t_lvl = lvl_ok ? price_level(n, p->V, lvl_visits) : 1e300;
        char pr[128];
        std::snprintf(pr, sizeof pr, " auto-price=fw:%.3gms,sparse:%.3gms,level:%.3gms", t_fw < 1e299 ? t_fw * 1e3 : -1.0,
                      t_sssp < 1e299 ? t_sssp * 1e3 : -1.0, t_lvl < 1e299 ? t_lvl * 1e3 : -1.0);
        auto_note = pr;
        if (fw_ok || sssp_ok || lvl_ok)
            algo = t_lvl <= std::min(t_fw, t_sssp) ? SRT_ALGO_LEVEL : t_sssp < t_fw ? SRT_ALGO_SSSP : SRT_ALGO_FW;
    }
    if (algo < 0) {
        const std::string why = want == SRT_ALGO_SSSP ? why_sssp
                                : want == SRT_ALGO_FW ? why_fw
                                : want == SRT_ALGO_LEVEL ? why_lvl
                                                         : why_fw + "; " + why_sssp;
        return fail(SRT_ERR_UNSUPPORTED, ("no exact path key for this graph: " + why).c_str());
    }
    p->algo = algo;
    if (algo == SRT_ALGO_LEVEL) {
        // levels are exact integers <= B in units of g: 2-byte download records
        // (quantized: B < 32 << sh < 2^31, 4-byte ones)
        p->kp.g = cs.gcd;
        p->kp.lmax = lvl_bound;
        p->kp.lat32 = true;
        p->key_type = p->lvl_q ? srt::KEY_U32 : srt::KEY_U16;
        f16 = false;

    } else {
        p->lvl_q = 0;
        p->lvl_sym = p->lvl_sym_lat = false;
        (void)hipFree(p->d_lat16);
        p->d_lat16 = nullptr;
        // the level probe's class CSRs (sized for it): freed before the
        // closure families size anything by the free HBM; their own runs grow
        // these arrays again from zero
        for (void *q : {(void *)p->d_tpk, (void *)p->d_tpk2, (void *)p->d_tcls, (void *)p->d_tccnt}) (void)hipFree(q);
        p->d_tpk = p->d_tpk2 = nullptr;
        p->d_tcls = p->d_tccnt = nullptr;
        p->t_cap = p->tcls_cap = p->lvl_cap = 0;
    }
    // SSSP plans read their in-edges (with loss) from the host-built list, never
    // d_loss: drop the deferred upload so run_tail does not copy it
    if (algo == SRT_ALGO_SSSP) {
        p->h_loss_defer = nullptr;
        if (defer_loss && srt::first_bad_loss(g) != ~0ull)  // no device check on this path
            return fail(SRT_ERR_INVALID, "Edge 'packet_loss' is not in the range [0,1]");
    }
    p->row0 = 0;
    p->row1 = n;
    p->rows_alloc = n;
    char d[200];
    if (algo == SRT_ALGO_LEVEL) {
        if (p->lvl_q)
            std::snprintf(d, sizeof d, "level:u32 g=%llu q=%u lmax=%llu(probe) V=%u n=%u visits=%llu loss=in-solve%s",
                          (unsigned long long)p->kp.g, p->lvl_q, (unsigned long long)p->kp.lmax, p->V, n,
                          (unsigned long long)lvl_visits, p->lvl_sym ? (p->d_lat16 ? " rows=sym lat16" : " rows=sym") : "");
        else
            std::snprintf(d, sizeof d, "level:u16 g=%llu lmax=%llu(probe) V=%u n=%u visits=%llu loss=in-solve%s",
                          (unsigned long long)p->kp.g, (unsigned long long)p->kp.lmax, p->V, n,
                          (unsigned long long)lvl_visits, p->lvl_sym ? (p->d_lat16 ? " rows=sym lat16" : " rows=sym") : "");
    } else if (algo == SRT_ALGO_FW) {
        p->fw_f16 = f16 && p->fw_glds;
        if (const char *e = std::getenv("SRT_FW_P1")) p->fw_p1 = std::atoi(e);
        if (const char *e = std::getenv("SRT_FW_EMULATE_RANKS")) p->emulate_ranks = (uint32_t)std::atoi(e);
        if (p->emulate_ranks > 1) {
            // emulated rank 0 owns the first max(1, blocks / N) block-rows (fw_rounds_t)
            const uint32_t nblk = p->Vp / srt::FW_B;
            const uint32_t rows_per = std::max<uint32_t>(1, nblk / p->emulate_ranks) * srt::FW_B;
            if (srt_status st = build_loss_rows(p, (int)p->emulate_ranks, rows_per, err); st != SRT_OK) {
                srt_plan_destroy(p);
                return st;
            }
        }
        if (const char *e = std::getenv("SRT_FW_BAND")) p->fw_band = e[0] == '1';
        std::snprintf(d, sizeof d, "fw:%s B=%d g=%llu lmax=%llu%s V=%u n=%u stage=%s band=%d loss=tight-dag%s",
                      p->fw_f16                     ? "f16key"
                      : p->key_type == srt::KEY_U16 ? "u16key"
                      : p->key_type == srt::KEY_U32 ? "u32key"
                      : p->key_type == srt::KEY_F64 ? "f64key"
                                                    : "u64key",
                      srt::FW_B, (unsigned long long)p->kp.g, (unsigned long long)p->kp.lmax,
                      cs.complete ? "(complete)" : ecc_units != ~0ull && ecc_units == p->kp.lmax ? "(ecc)" : "(V-1)",
                      p->V, n,
                      p->fw_glds ? "glds" : "reg", (int)p->fw_band, p->kp.lat32 ? "/u32" : "/u64");
    } else {
        // R words of 64 sources per lane (one wave walks a vertex's in-edges
        // once for 64*R sources), and as many groups in flight as ~256 MB of
        // path state allows (Infinity Cache sized), never more than the rows need
        const uint32_t words = std::max<uint32_t>(1, (n + 63) / 64);
        // Many groups in flight amortise each sweep's launch and latency chain
        // and the convergence tail (C4, measured: 192 MB of path state 3.0 s,
        // 1.6 GB 1.73 s, 6.4 GB 1.53 s, 12.8 GB 1.49 s), capped at 1/8 of the
        // free HBM.
        uint64_t budget_mb = 6400;
        size_t free_b = 0, total_b = 0;
        if (hipMemGetInfo(&free_b, &total_b) == hipSuccess && free_b)
            budget_mb = std::max<uint64_t>(64, std::min<uint64_t>(budget_mb, (free_b >> 20) / 8));
        const uint32_t R = words >= 4 ? 4 : words >= 2 ? 2 : 1;
        const uint64_t per_group = (uint64_t)p->V * 64 * 8 * R;
        uint64_t G = std::max<uint64_t>(1, (budget_mb << 20) / std::max<uint64_t>(per_group, 1));
        G = std::min<uint64_t>(G, (words + R - 1) / R);
        G = std::min<uint64_t>(G, 256);
        p->sssp_r = R;
        p->sssp_nb = (uint32_t)(G * R);
        p->n_in_edges = n_in;
        d[0] = '\0';  // named once the bucket width is known (below)
    }
    p->desc = d;
    tr.mark("create: key/algo choice");

    // 4. the family's buffers; self-loop values
    srt_status st;
    hipError_t e;
#define PLAN_TRY(x)                \
    do {                           \
        st = (x);                  \
        if (st != SRT_OK) {        \
            srt_plan_destroy(p);   \
            return st;             \
        }                          \
    } while (0)
    if (algo == SRT_ALGO_FW)
        PLAN_TRY(dmalloc(reinterpret_cast<uint8_t **>(&p->d_D), (size_t)p->Vp * p->Vp * srt::key_bytes(p->key_type),
                         err));
    PLAN_TRY(dmalloc(&p->d_out_lat, (size_t)n * n, err));
    PLAN_TRY(dmalloc(&p->d_out_loss, (size_t)n * n, err));
    if (algo == SRT_ALGO_SSSP) {
        std::vector<uint64_t> in_ptr;
        std::vector<srt::InEdge> in_edge;
        build_in_edges(g, p->sssp_g, n_in, &in_ptr, &in_edge);
        // latency-first frontier sweeps (srt_frontier.hip) when every finite
        // distance fits u16 units: the proved bound (eccentricity, or (V-1) *
        // max edge) below 0xFFFF.  Knob SRT_SSSP_KEY=64 keeps the packed-key
        // sweep (A/B, tests).
        {
            const uint64_t maxu = cs.maxlat / cs.gcd;
            const unsigned __int128 lb = ecc_units != ~0ull ? (unsigned __int128)ecc_units
                                                            : (unsigned __int128)(p->V ? p->V - 1 : 0) * maxu;
            const char *kk = std::getenv("SRT_SSSP_KEY");
            p->sssp_frontier = lb < 0xffff && !(kk && std::atoi(kk) == 64);
        }
        PLAN_TRY(dmalloc(&p->d_in_ptr, in_ptr.size(), err));
        PLAN_TRY(dmalloc(&p->d_in_edge, in_edge.size(), err));
        // source order of the sweep's words (knob SRT_SSSP_ORDER=0: table order)
        {
            const char *ko = std::getenv("SRT_SSSP_ORDER");
            const int om = ko ? std::atoi(ko) : 1;
            // 1: launches in breadth-first order, rows within a launch in
            // shortest-latency-tree level order (frontier sweeps); 2: breadth-first
            // only; 3: tree level order only (A/B)
            if (om == 1 || om == 2) p->h_bfs_rank = hop_rank(g);
            if (om == 3) p->h_bfs_rank = spt_rank(g);
            if (om == 1 && p->sssp_frontier) p->h_spt_rank = spt_rank(g);  // read by frontier sweeps only
        }
        if (!p->sssp_frontier) {
            PLAN_TRY(dmalloc(&p->d_sD, (size_t)p->sssp_nb * p->V * 64, err));
            PLAN_TRY(dmalloc(&p->d_smask, (size_t)2 * p->sssp_nb * p->V, err));
            PLAN_TRY(dmalloc(&p->d_sflag, (size_t)12 * p->sssp_nb, err));  // flags + delta-stepping ring
            PLAN_TRY(dmalloc(&p->d_spend, (size_t)p->sssp_nb * p->V, err));
        }
        {
            // delta-stepping bucket width = SRT_SSSP_DELTA x the mean in-edge
            // latency (units of g); default 0 = ungated sweeps, the faster on
            // C4 (100k BA, one GPU: ungated 1.60 s, factor 0.25 / 1.0 1.68 s --
            // fewer relaxations but not fewer gathered lines)
            double f = 0.0;
            if (const char *ev = std::getenv("SRT_SSSP_DELTA")) f = std::atof(ev);
            double sum = 0.0;
            for (const srt::InEdge &ie : in_edge) sum += ie.w;
            const double mean = in_edge.empty() ? 0.0 : sum / (double)in_edge.size();
            p->sssp_delta = f > 0.0 ? (uint32_t)std::max(1.0, std::min(mean * f, 1e9)) : 0u;
            // sweep bound: V + 2 Bellman-Ford sweeps once the threshold passes
            // the longest simple path, plus the sweeps it takes to get there
            uint64_t wmax = 0;
            for (const srt::InEdge &ie : in_edge) wmax = std::max<uint64_t>(wmax, ie.w);
            p->sssp_tmax = (uint64_t)p->V + 4;
            if (p->sssp_delta) p->sssp_tmax += (uint64_t)p->V * wmax / p->sssp_delta + 2;
        }
        char dd[256];
        std::snprintf(dd, sizeof dd, "sssp:lat32|f32 g=%llu V=%u n=%u E_in=%llu R=%u groups=%u delta=%u order=%s",
                      (unsigned long long)p->sssp_g, p->V, p->n, (unsigned long long)p->n_in_edges, p->sssp_r,
                      p->sssp_nb / p->sssp_r, p->sssp_delta, p->h_bfs_rank.empty() ? "table" : "bfs");
        p->desc = dd;
        if (const char *ev = std::getenv("SRT_SSSP_ACT")) {
            const int k = std::atoi(ev);
            p->sssp_act_on = k != 0;
            p->sssp_act_from = k > 1 ? (uint32_t)k : 0u;
        }
        if (p->sssp_frontier) {
            // blocks in flight: as many as half the free HBM holds (C4: ~0.7 GB a
            // block, capped at 64 = 32k sources), never more than the rows need;
            // knob SRT_SSSP_FR_NB (measurement)
            const uint64_t bb = srt::frontier_block_bytes(p->V, n_in);
            size_t free_b = 0, total_b = 0;
            uint64_t nb = 64;
            if (hipMemGetInfo(&free_b, &total_b) == hipSuccess && free_b)
                nb = std::min<uint64_t>(nb, std::max<uint64_t>(1, (free_b / 2) / std::max<uint64_t>(bb, 1)));
            // launches of equal size (C4: 196 blocks as 4 x 49, not 64+64+64+4 --
            // a small last launch pays a full run of sweeps: 0.70 -> 0.68 s)
            const uint64_t blocks_all = std::max<uint32_t>(1, (n + 511) / 512);
            nb = (blocks_all + (blocks_all + nb - 1) / nb - 1) / ((blocks_all + nb - 1) / nb);
            if (const char *ev = std::getenv("SRT_SSSP_FR_NB")) nb = std::max<uint64_t>(1, std::atoll(ev));
            nb = std::min<uint64_t>(nb, blocks_all);
            p->fr_nb = (uint32_t)nb;
            int cus = 256;
            (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, p->device);
            p->fr_grid = (uint32_t)std::max(1, cus) * 8;
            if (const char *ev = std::getenv("SRT_SSSP_FR_GRID")) p->fr_grid = (uint32_t)std::max(1, std::atoi(ev));
            // undirected (latency-symmetric) graphs: L(s, v) = L(v, s), so every
            // launch starts from the exact columns of the earlier launches' rows
            // (srt_frontier.hip fr_sym_copy_kernel) -- which needs the latencies
            // of all rows resident: n * V * 2 B (C4: 20 GB), if a quarter of the
            // free HBM holds them.  Knob SRT_SSSP_SYM=0 (A/B, tests).
            const uint64_t all_blocks = std::max<uint32_t>(1, (n + 511) / 512);
            const char *ks = std::getenv("SRT_SSSP_SYM");
            p->fr_symg = latency_symmetric(g, in_ptr, in_edge, cs.gcd);
            p->fr_sym = !(ks && std::atoi(ks) == 0) && all_blocks > nb &&
                        all_blocks * p->V * 1024ull <= (uint64_t)free_b / 4 && p->fr_symg;
            // a smaller first launch: the only one whose latency phase starts
            // from the sources alone (C4, 4 launches: 49+49+49+49 blocks 0.488 s,
            // 12+61+61+62 0.463, 20+... 0.465, 28+... 0.463); ~1/12 of the
            // blocks, the rest keep the launch count, so their buffers grow to
            // hold them.  Knob SRT_FR_FIRST = blocks (0: equal launches; A/B).
            p->fr_first = 0;
            if (p->fr_sym) {
                const char *ev = std::getenv("SRT_FR_FIRST");
                const uint64_t f = ev ? std::atoll(ev) : all_blocks / 12, k = (all_blocks + nb - 1) / nb;
                if (f > 0 && f < nb && k >= 2) {
                    const uint64_t rest = (all_blocks - f + k - 2) / (k - 1);
                    if (rest <= 64 && rest * bb <= free_b / 2) {
                        nb = std::max(nb, rest);
                        p->fr_first = (uint32_t)f;
                        p->fr_nb = (uint32_t)nb;
                    }
                }
            }
            p->fr_lblocks = p->fr_sym ? (uint32_t)all_blocks : (uint32_t)nb;
            PLAN_TRY(dmalloc(&p->d_fl, (size_t)p->fr_lblocks * p->V * 512, err));
            PLAN_TRY(dmalloc(&p->d_fp, (size_t)nb * p->V * 512, err));
            PLAN_TRY(dmalloc(&p->d_ftight, (size_t)nb * std::max<uint64_t>(n_in, 1) * 64, err));
            PLAN_TRY(dmalloc(&p->d_fce, (size_t)nb * std::max<uint64_t>(n_in, 1), err));
            PLAN_TRY(dmalloc(&p->d_fcnt, (size_t)nb * p->V, err));
            PLAN_TRY(dmalloc(&p->d_fctl, 8, err));
            PLAN_TRY(dmalloc(reinterpret_cast<uint8_t **>(&p->d_fchg), (size_t)nb * p->V * srt::frontier_chg_bytes(), err));
            PLAN_TRY(dmalloc(&p->d_fact, (size_t)nb * p->V, err));
            PLAN_TRY(dmalloc(&p->d_fsb, (size_t)2 * nb * p->V * 64, err));
            PLAN_TRY(dmalloc(&p->d_ffin, (size_t)nb * p->V, err));
            PLAN_TRY(dmalloc(&p->d_fimp, 1, err));
            if ((e = hipMemsetAsync(p->d_fchg, 0, (size_t)nb * p->V * srt::frontier_chg_bytes(), p->stream)) != hipSuccess ||
                (e = hipMemsetAsync(p->d_fact, 0, (size_t)nb * p->V * 4, p->stream)) != hipSuccess ||
                (e = hipMemsetAsync(p->d_fimp, 0, 4, p->stream)) != hipSuccess ||
                (e = hipHostMalloc((void **)&p->h_fimp, 4, 0)) != hipSuccess) {
                srt_plan_destroy(p);
                return hip_fail(err, e, "sparse frontier buffers");
            }
            p->fr_t = 1;
            char df[160];
            std::snprintf(df, sizeof df,
                          "sssp:frontier u16|f32 g=%llu lmax=%llu%s V=%u n=%u E_in=%llu blocks=%u first=%u order=%s seed=%s",
                          (unsigned long long)p->sssp_g, (unsigned long long)(ecc_units != ~0ull ? ecc_units : 0),
                          ecc_units != ~0ull ? "(ecc)" : "(V-1)", p->V, p->n, (unsigned long long)p->n_in_edges,
                          p->fr_nb, p->fr_first,
                          p->h_bfs_rank.empty() ? "table" : p->h_spt_rank.empty() ? "bfs" : "bfs+tree",
                          p->fr_sym ? "sym" : "none");
            p->desc = df;
        }
        if (p->sssp_act_on && !p->sssp_frontier)
            PLAN_TRY(dmalloc(&p->d_sact, (size_t)3 * (p->sssp_nb / p->sssp_r) * p->V, err));
        if ((e = hipHostMalloc((void **)&p->h_sflag, (size_t)p->sssp_nb * sizeof(uint32_t), 0)) != hipSuccess) {
            srt_plan_destroy(p);
            return hip_fail(err, e, "hipHostMalloc");
        }
        if (p->sssp_frontier) {
            // Hub-spreading vertex order for the frontier sweeps: a wave works
            // through a 64-vertex chunk item by item, so a chunk of hubs (BA
            // graphs number them first: C4's vertices 0..63 have ~1000
            // in-edges each) would keep one wave busy for the whole sweep
            // (measured: C4 1.71 s -> 1.07 s with the hubs dealt out).  The
            // cpb highest in-degree vertices go to slot 0 of the cpb chunks,
            // one each; every other vertex keeps its relative order (BA graphs'
            // id locality: neighbours of similar age gather similar rows).
            const uint32_t V = p->V, cpb = (V + 63) / 64;
            std::vector<uint32_t> order(V), pi(V, ~0u);
            for (uint32_t v = 0; v < V; ++v) order[v] = v;
            std::stable_sort(order.begin(), order.end(), [&](uint32_t a, uint32_t b) {
                return in_ptr[a + 1] - in_ptr[a] > in_ptr[b + 1] - in_ptr[b];
            });
            // (measured, C4: no hubs dealt 1.30 s, the top 64 0.95 s, one per chunk 0.80 s)
            const uint32_t H = V >= 64 * cpb ? cpb : (V > cpb ? cpb - 1 : 0);  // chunks with a full slot 0
            std::vector<uint8_t> hub(V, 0);
            for (uint32_t h = 0; h < H; ++h) {
                pi[order[h]] = h * 64;
                hub[order[h]] = 1;
            }
            for (uint32_t v = 0, pos = 0; v < V; ++v) {
                if (hub[v]) continue;
                while (pos % 64 == 0 && pos / 64 < H) ++pos;  // slot 0 of a hub chunk
                pi[v] = pos++;
            }
            std::vector<uint64_t> ip(V + 1, 0), op(V + 1, 0);
            for (uint32_t v = 0; v < V; ++v) {
                ip[pi[v] + 1] = in_ptr[v + 1] - in_ptr[v];
                uint64_t d = 0;
                for (uint64_t k = g->row_ptr[v]; k < g->row_ptr[v + 1]; ++k) d += g->col[k] != v;
                op[pi[v] + 1] = d;
            }
            for (uint32_t v = 0; v < V; ++v) {
                ip[v + 1] += ip[v];
                op[v + 1] += op[v];
            }
            std::vector<srt::InEdge> ie(in_edge.size());
            std::vector<uint32_t> oc(std::max<uint64_t>(op[V], 1));
            for (uint32_t v = 0; v < V; ++v) {
                uint64_t o = ip[pi[v]];
                for (uint64_t k = in_ptr[v]; k < in_ptr[v + 1]; ++k, ++o) {
                    ie[o] = in_edge[k];
                    ie[o].u = pi[in_edge[k].u];
                }
                o = op[pi[v]];
                for (uint64_t k = g->row_ptr[v]; k < g->row_ptr[v + 1]; ++k)
                    if (g->col[k] != v) oc[o++] = pi[g->col[k]];
            }
            in_ptr.swap(ip);
            in_edge.swap(ie);
            p->h_fnodes.resize(n);
            for (uint32_t i = 0; i < n; ++i) p->h_fnodes[i] = pi[nodes[i]];
            PLAN_TRY(dmalloc(&p->d_fnodes, std::max<uint32_t>(n, 1), err));
            PLAN_TRY(dmalloc(&p->d_frow_ptr, op.size(), err));
            PLAN_TRY(dmalloc(&p->d_fcol, oc.size(), err));
            if ((e = hipMemcpy(p->d_fnodes, p->h_fnodes.data(), (size_t)n * 4, hipMemcpyHostToDevice)) != hipSuccess ||
                (e = hipMemcpy(p->d_frow_ptr, op.data(), op.size() * 8, hipMemcpyHostToDevice)) != hipSuccess ||
                (e = hipMemcpy(p->d_fcol, oc.data(), oc.size() * 4, hipMemcpyHostToDevice)) != hipSuccess) {
                srt_plan_destroy(p);
                return hip_fail(err, e, "upload frontier graph");
            }
        }
        if ((e = hipMemcpy(p->d_in_ptr, in_ptr.data(), in_ptr.size() * 8, hipMemcpyHostToDevice)) != hipSuccess ||
            (e = hipMemcpy(p->d_in_edge, in_edge.data(), in_edge.size() * sizeof(srt::InEdge),
                           hipMemcpyHostToDevice)) != hipSuccess) {
            srt_plan_destroy(p);
            return hip_fail(err, e, "upload in-edges");
        }
    }
#undef PLAN_TRY
    p->h_sl_lat = std::move(sl_lat);
    p->h_sl_loss = std::move(sl_loss);
    if ((n && (e = hipMemcpyAsync(p->d_sl_lat, p->h_sl_lat.data(), (size_t)n * 8, hipMemcpyHostToDevice,
                                  p->stream)) != hipSuccess) ||
        (n && (e = hipMemcpyAsync(p->d_sl_loss, p->h_sl_loss.data(), (size_t)n * 4, hipMemcpyHostToDevice,
                                  p->stream)) != hipSuccess) ||
        (e = hipStreamSynchronize(p->stream)) != hipSuccess) {
        srt_plan_destroy(p);
        return hip_fail(err, e, "upload");
    }
    tr.mark("create: upload");
    p->desc += auto_note;
    p->in_create = false;
    p->create_device_ms = 0.0;
    for (size_t i = 0; i + 1 < p->cspan.size(); i += 2) {
        float ms = 0.f;
        if (hipEventElapsedTime(&ms, p->cspan[i], p->cspan[i + 1]) == hipSuccess) p->create_device_ms += ms;
    }
    for (hipEvent_t e : p->cspan) (void)hipEventDestroy(e);
    p->cspan.clear();
    *plan_out = p;
    return SRT_OK;
}

// The device build in two host phases: the closure (FW rounds / SSSP sweeps)
// is enqueued first, so that run_tail's blocking host work (the deferred
// loss upload) overlaps it on the GPU.
srt_status run_closure(srt_plan *p, srt_err *err) {
    HIP_TRY(hipSetDevice(p->device), "hipSetDevice");
    hipEventRecord(p->ev_begin, p->stream);
    p->loss_ms = 0.0;
    const int rank = p->comm ? p->comm->rank : 0;
    unsigned long long *rstats = p->comm ? p->d_rstats + 2 * rank : p->d_stats;
    if (p->algo == SRT_ALGO_SSSP) return srt::sssp_run(p, rstats, err);
    if (p->algo == SRT_ALGO_LEVEL) return SRT_OK;  // no closure: the rows are solved in run_tail (level_run)
    // N-rank emulation (measurement only): the first run closes D for
    // real; later runs replay rank 0's schedule on the closed D (every
    // round leaves a closed D unchanged, and the kernels' cost does not
    // depend on the keys), so rank 0's loss-pass share sees valid keys
    if (!p->emu_closed) srt::fw_init(p);
    if (!p->fw_sym_known) {
        if (!p->d_flag32) HIP_TRY(hipMalloc(&p->d_flag32, 4), "hipMalloc(flag)");
        if (srt_status st = srt::fw_sym_check(p, err); st != SRT_OK) return st;
    }
    return srt::fw_rounds(p, err);
}

// End-to-end build: the edge losses, uploaded while the closure runs and
// range-checked on the device (LossUpload).  The copies run on the host
// thread once their stream reaches them, so they go on the comm stream (idle
// on one GPU; the closure is all on the main and side streams) and the main
// stream waits for them before the loss pass -- on the main stream they would
// queue behind the closure (measured: C3 +19 ms, serial).
// Level plans (n_adj < 2^32): only the losses the class CSRs read cross PCIe
// -- their adjacency indices listed on the device (latency <= B units, not a
// self-loop: C3 5.4M of 268M entries), downloaded into the pinned staging,
// gathered on host threads and scattered into d_loss -- while the range check
// of every loss (the reference's parse-time error) runs on host threads
// behind the build (p->loss_checker, joined before h_lossbad is read).
// C3: the 1 GB loss upload (~25 ms on the critical path) becomes ~22 MB each
// way.  false: not applicable (the caller uploads everything).
bool upload_level_losses(srt_plan *p, srt_err *err, srt_status *st) {
    *st = SRT_OK;
    if (p->algo != SRT_ALGO_LEVEL || p->n_adj >= (1ull << 32) || !p->lvl_cap || std::getenv("SRT_LOSS_FULL"))
        return false;
    // the pinned staging: waited for when busy -- the first one-call build of
    // a process without srt_init pins it on a thread behind its closure
    // (build_e2e), and the needed-loss path (~5 ms at C3) beats the full
    // pageable upload it would otherwise fall back to (~25-48 ms)
    Trace tr;
    std::unique_lock<std::mutex> lk(g_pinned.m, std::try_to_lock);
    if (!lk.owns_lock()) {
        lk.lock();
        tr.mark("losses: waited for the pinned staging");
    }
    const uint64_t cap = p->lvl_cap;  // the probe's count: >= the run's (its bound is >= B)
    if (g_pinned.bytes < 64) {
        tr.mark("losses: no pinned staging, full upload");
        return false;
    }
    hipStream_t M = p->stream;
    auto fail = [&](hipError_t e, const char *what) {
        *st = hip_fail(err, e, what);
        return true;
    };
    hipError_t e = hipSuccess;
    if (!p->d_lidx || p->lidx_cap < cap) {
        (void)hipFree(p->d_lidx);
        p->d_lidx = nullptr;
        e = hipMalloc(&p->d_lidx, cap * 8 + 32);
        if (e != hipSuccess) return fail(e, "hipMalloc(loss indices)");
        p->lidx_cap = cap;
    }
    uint32_t *d_idx = reinterpret_cast<uint32_t *>(p->d_lidx);
    float *d_val = reinterpret_cast<float *>(d_idx + cap);
    unsigned long long *d_cnt = reinterpret_cast<unsigned long long *>(d_val + cap + (cap & 1));
    srt::level_loss_index(p, d_idx, cap, d_cnt, M);
    uint64_t *h = reinterpret_cast<uint64_t *>(g_pinned.buf);
    e = hipMemcpyAsync(h, d_cnt, 8, hipMemcpyDeviceToHost, M);
    if (e == hipSuccess) e = hipStreamSynchronize(M);
    if (e != hipSuccess) return fail(e, "loss indices (count)");
    const uint64_t cnt = h[0];
    tr.mark("losses: needed entries listed");
    // (cnt > cap cannot happen: the probe's bound is >= the run's)
    if (cnt > cap || g_pinned.bytes < cnt * 8) {  // the full upload
        tr.mark("losses: staging too small, full upload");
        return false;
    }
    // the range check of every loss, behind the build (8 host threads),
    // started once the needed losses are gathered (knob SRT_LOSSCHK_EARLY=1:
    // before the gather, A/B) -- it streams the whole loss array, and the
    // gather's cache misses wait behind it
    const float *src = p->h_loss_defer;
    const uint64_t m = p->n_adj;
    unsigned long long *hb = p->h_lossbad;
    *hb = ~0ull;
    auto start_checker = [&]() {
        p->loss_checker = std::thread([src, m, hb] {
            const int T = std::max(1, std::min(8, host_threads(m)));
            std::vector<uint64_t> first(T, ~0ull);
            std::vector<std::thread> pool;
            const uint32_t *q = reinterpret_cast<const uint32_t *>(src);
            for (int t = 0; t < T; ++t)
                pool.emplace_back([&, t] {
                    for (uint64_t k = m * t / T; k < m * (t + 1) / T; ++k)
                        if (srt::loss_bits_bad(q[k])) {
                            first[t] = k;
                            break;
                        }
                });
            for (auto &th : pool) th.join();
            *hb = *std::min_element(first.begin(), first.end());
        });
    };
    const bool early = std::getenv("SRT_LOSSCHK_EARLY") && std::atoi(std::getenv("SRT_LOSSCHK_EARLY")) == 1;
    if (early) start_checker();
    uint32_t *hidx = reinterpret_cast<uint32_t *>(g_pinned.buf);
    float *hval = reinterpret_cast<float *>(hidx + cnt);
    e = hipMemcpyAsync(hidx, d_idx, cnt * 4, hipMemcpyDeviceToHost, M);
    if (e == hipSuccess) e = hipStreamSynchronize(M);
    if (e != hipSuccess) return fail(e, "loss indices");
    tr.mark("losses: indices on the host");
    {
        const int T = host_threads(cnt * 16);
        std::vector<std::thread> pool;
        // one cache miss a loss (~330 scattered columns a row): 32 gathers
        // ahead in flight by prefetch
        auto part = [&](int t) {
            const uint64_t a = cnt * t / T, b = cnt * (t + 1) / T;
            for (uint64_t i = a; i < b; ++i) {
                if (i + 32 < b) __builtin_prefetch(src + hidx[i + 32], 0, 0);
                hval[i] = src[hidx[i]];
            }
        };
        for (int t = 1; t < T; ++t) pool.emplace_back(part, t);
        part(0);
        for (auto &th : pool) th.join();
    }
    tr.mark("losses: gathered");
    if (!early) start_checker();
    e = hipMemcpyAsync(d_val, hval, cnt * 4, hipMemcpyHostToDevice, M);
    if (e != hipSuccess) return fail(e, "upload (needed losses)");
    srt::loss_scatter(d_idx, d_val, cnt, p->d_loss, M);
    // symmetric plans (identity rows, latencies checked at create): every
    // uploaded loss must equal its mirror's, else the run builds its in-rows
    uint32_t *d_ok = reinterpret_cast<uint32_t *>(d_cnt + 1);
    if (p->lvl_sym) {
        h[0] = 1;
        e = hipMemcpyAsync(d_ok, h, 4, hipMemcpyHostToDevice, M);
        if (e == hipSuccess) srt::loss_mirror_check(d_idx, cnt, p->V, p->d_loss, d_ok, M);
        if (e == hipSuccess) e = hipMemcpyAsync(h, d_ok, 4, hipMemcpyDeviceToHost, M);
    }
    // the staging is reused by the download: the upload must be done first
    if (e == hipSuccess) e = hipStreamSynchronize(M);
    if (e != hipSuccess) return fail(e, "upload (needed losses)");
    if (p->lvl_sym && reinterpret_cast<uint32_t *>(h)[0] == 0) p->lvl_sym = false;
    tr.mark("losses: uploaded, scattered, mirror-checked");
    p->h_loss_defer = nullptr;
    return true;
}

void join_loss_check(srt_plan *p) {
    if (p->loss_checker.joinable()) p->loss_checker.join();
}

srt_status upload_deferred_loss(srt_plan *p, srt_err *err) {
    if (p->h_loss_defer && !p->d_lossbad) {
        HIP_TRY(hipMalloc(&p->d_lossbad, 8), "hipMalloc(loss check)");
        HIP_TRY(hipHostMalloc((void **)&p->h_lossbad, 8, 0), "hipHostMalloc(loss check)");
    }
    if (p->h_loss_defer) {
        srt_status st;
        if (upload_level_losses(p, err, &st)) return st;
        p->lvl_sym = false;  // the losses' mirrors were not checked: build the in-rows
    }
    if (p->h_loss_defer) {
        hipStream_t up = p->comm ? p->stream : p->comm_stream;
        if (!p->d_lossbad) {
            HIP_TRY(hipMalloc(&p->d_lossbad, 8), "hipMalloc(loss check)");
            HIP_TRY(hipHostMalloc((void **)&p->h_lossbad, 8, 0), "hipHostMalloc(loss check)");
        }
        *p->h_lossbad = ~0ull;
        {
            LossUpload lu;
            lu.src = p->h_loss_defer;
            lu.m = p->n_adj;
            if (srt_status s2 = lu.run(p, up, err); s2 != SRT_OK) return s2;
        }
        HIP_TRY(hipMemcpyAsync(p->h_lossbad, p->d_lossbad, 8, hipMemcpyDeviceToHost, up), "download (loss check)");
        if (up != p->stream) {
            if (!p->ev_upload) HIP_TRY(hipEventCreateWithFlags(&p->ev_upload, hipEventDisableTiming), "event");
            HIP_TRY(hipEventRecord(p->ev_upload, up), "event record");
            HIP_TRY(hipStreamWaitEvent(p->stream, p->ev_upload, 0), "event wait");
        }
        p->h_loss_defer = nullptr;
    }
    return SRT_OK;
}

srt_status run_tail(srt_plan *p, srt_err *err) {
    srt_status st;
    // table rows [row0, row1) of this rank; every rank then holds the whole
    // table after the row exchange, and the stats of all ranks
    const int rank = p->comm ? p->comm->rank : 0, nranks = p->comm ? p->comm->nranks : 1;
    unsigned long long *rstats = p->comm ? p->d_rstats + 2 * rank : p->d_stats;
    if ((st = upload_deferred_loss(p, err)) != SRT_OK) return st;
    if (p->algo != SRT_ALGO_SSSP) {
        // exact loss over the tight DAG (sharded: over this rank's own
        // closure rows, see fw_loss)
        st = srt::fw_loss(p, rstats, err);
        if (st != SRT_OK) return st;
        if (!p->comm && p->emulate_ranks > 1) p->emu_closed = true;
    }
    if (!p->comm && p->shard_tail) {
        if (!p->tail_expanded) srt::expand_shard_rows(p, (int)p->emulate_ranks);  // emulation: stale slots
    } else if (p->comm && p->shard_tail) {
        // the staged rows (latency units and / or f32 loss per pair) were
        // all-gathered chunk by chunk behind the fold, and every rank expanded
        // each chunk into its table behind its all-gather (fw_loss)
        if ((st = srt::comm_allgather_inplace(p->comm, p->d_rstats, 16, p->stream, err)) != SRT_OK) return st;
        if (!p->tail_expanded) srt::expand_shard_rows(p, nranks);
        srt::reduce_rank_stats(p, nranks);
    } else if (p->comm) {
        const size_t per = (size_t)p->rows_alloc / nranks * p->n;
        if ((st = srt::comm_allgather_inplace(p->comm, p->d_out_lat, per * 8, p->stream, err)) != SRT_OK ||
            (st = srt::comm_allgather_inplace(p->comm, p->d_out_loss, per * 4, p->stream, err)) != SRT_OK ||
            (st = srt::comm_allgather_inplace(p->comm, p->d_rstats, 16, p->stream, err)) != SRT_OK)
            return st;
        srt::reduce_rank_stats(p, nranks);
    }
    hipEventRecord(p->ev_end, p->stream);
    HIP_TRY(hipGetLastError(), "kernel launch");
    p->ran = true;
    return SRT_OK;
}
}  // namespace

srt_status srt_plan_run_async(srt_plan *p, srt_err *err) {
    clear_err(err);
    if (!p) {
        set_err(err, SRT_ERR_INVALID, "null plan");
        return SRT_ERR_INVALID;
    }
    ++p->run_no;  // the packet stage's packed table is stale from here
    srt_status st = run_closure(p, err);
    if (st == SRT_OK) st = run_tail(p, err);
    return st;
}

srt_status srt_plan_sync(srt_plan *p, srt_err *err) {
    clear_err(err);
    if (!p) {
        set_err(err, SRT_ERR_INVALID, "null plan");
        return SRT_ERR_INVALID;
    }
    HIP_TRY(hipStreamSynchronize(p->stream), "hipStreamSynchronize");
    // collect timings
    float ms = 0.f;
    p->total_ms = 0.0;
    if (hipEventElapsedTime(&ms, p->ev_begin, p->ev_end) == hipSuccess) p->total_ms = ms;
    p->p3_ms = 0.0;
    for (uint64_t i = 0; i < p->p3_launches; ++i) {
        if (hipEventElapsedTime(&ms, p->ev[2 * i], p->ev[2 * i + 1]) == hipSuccess) p->p3_ms += ms;
    }
    if (p->algo != SRT_ALGO_SSSP && p->ev_loss0 && hipEventElapsedTime(&ms, p->ev_loss0, p->ev_loss1) == hipSuccess)
        p->loss_ms = ms;
    if (p->algo == SRT_ALGO_LEVEL && p->d_lvisit) {
        unsigned long long v = 0;
        if (hipMemcpy(&v, p->d_lvisit, sizeof v, hipMemcpyDeviceToHost) == hipSuccess) p->lvl_visits = v;
    }
    // in-process transport: what this rank received matched its senders'
    // checksums (srt_comm.cpp local_collective)
    if (p->comm && srt::local_corrupt(p->comm)) {
        set_err(err, SRT_ERR_COMM,
                "in-process collective: data received from a peer device differs from the sender's (checksum)");
        return SRT_ERR_COMM;
    }
    return SRT_OK;
}

srt_status srt_plan_run(srt_plan *p, srt_err *err) {
    srt_status s = srt_plan_run_async(p, err);
    if (s != SRT_OK) return s;
    return srt_plan_sync(p, err);
}

srt_status srt_plan_fetch(srt_plan *p, srt_path *out, uint64_t *min_latency_ns, srt_err *err) {
    clear_err(err);
    Trace tr;
    if (!p || !p->ran) {
        set_err(err, SRT_ERR_INVALID, "plan has not been run");
        return SRT_ERR_INVALID;
    }
    HIP_TRY(hipSetDevice(p->device), "hipSetDevice");
    unsigned long long stats[2];
    HIP_TRY(hipMemcpyAsync(stats, p->d_stats, sizeof stats, hipMemcpyDeviceToHost, p->stream), "stats");
    HIP_TRY(hipStreamSynchronize(p->stream), "sync");
    if (stats[1] != 0) {
        // the reference panics in assert_eq!(paths.len(), nodes.len().pow(2))
        // (mod.rs:219); this is Rust 1.76's assert_eq! panic message
        char buf[200];
        const unsigned long long nn = (unsigned long long)p->n * p->n;
        std::snprintf(buf, sizeof buf, "assertion `left == right` failed\n  left: %llu\n right: %llu",
                      nn - stats[1], nn);
        set_err(err, SRT_ERR_DISCONNECTED, buf);
        return SRT_ERR_DISCONNECTED;
    }
    if (min_latency_ns) *min_latency_ns = stats[0];
    if (out && p->row_shard) {
        set_err(err, SRT_ERR_INVALID, "row-sharded plan: only its own rows were built (read them via srt_plan_table)");
        return SRT_ERR_INVALID;
    }
    if (out && p->n) {
        // AoS staging in chunks of at most 64 Mi entries (1 GiB): the 100k-node
        // table is 1e10 entries and must not be duplicated whole in HBM
        const uint64_t total = (uint64_t)p->n * p->n;
        const uint64_t chunk = std::min<uint64_t>(total, 1ull << 26);
        if (!p->d_pack) {
            void *ptr = nullptr;
            hipError_t e = hipMalloc(&ptr, chunk * sizeof(srt_path));
            if (e != hipSuccess) return hip_fail(err, e, "hipMalloc(pack)");
            p->d_pack = (srt_path *)ptr;
        }
        for (uint64_t off = 0; off < total; off += chunk) {
            const uint64_t c = std::min<uint64_t>(chunk, total - off);
            srt::pack_paths(p, off, c, p->d_pack, p->stream);
            HIP_TRY(hipMemcpyAsync(out + off, p->d_pack, c * sizeof(srt_path), hipMemcpyDeviceToHost, p->stream),
                    "download");
            HIP_TRY(hipStreamSynchronize(p->stream), "sync");
        }
    }
    tr.mark("fetch: pack+download");
    return SRT_OK;
}

srt_status srt_plan_table(srt_plan *p, uint64_t **d_lat, float **d_loss, uint32_t *n) {
    if (!p) return SRT_ERR_INVALID;
    if (d_lat) *d_lat = p->d_out_lat;
    if (d_loss) *d_loss = p->d_out_loss;
    if (n) *n = p->n;
    return SRT_OK;
}

const char *srt_plan_describe(const srt_plan *p) { return p ? p->desc.c_str() : ""; }

void *srt_plan_stream(srt_plan *p) { return p ? (void *)p->stream : nullptr; }

srt_status srt_plan_kernel_stats(const srt_plan *p, double *dominant_ms, uint64_t *launches,
                                 double *dominant_work, double *total_ms) {
    if (!p) return SRT_ERR_INVALID;
    if (dominant_ms) *dominant_ms = p->p3_ms;
    if (launches) *launches = p->p3_launches;
    if (dominant_work) *dominant_work = p->p3_work;
    if (total_ms) *total_ms = p->total_ms;
    return SRT_OK;
}

srt_status srt_plan_timing(const srt_plan *p, srt_timing *o) {
    if (!p || !o) return SRT_ERR_INVALID;
    o->total_ms = p->total_ms;
    o->dominant_ms = p->p3_ms;
    o->dominant_launches = p->p3_launches;
    o->dominant_work = p->p3_work;
    o->loss_ms = p->loss_ms;
    o->tight_edges = p->algo != SRT_ALGO_SSSP ? p->t_edges : 0;  // level solve: the pruned edges
    o->sharded_tail = p->algo != SRT_ALGO_SSSP && p->shard_tail ? 1u : 0u;  // dense: staged rows all-gathered
    o->sparse_split = 0u;  // the split sweep was removed (reserved)
    o->sparse_sweeps = p->algo == SRT_ALGO_SSSP ? p->sssp_sweeps : 0;
    o->loss_fold = p->algo == SRT_ALGO_FW && p->t_level ? 1u : 0u;
    o->reserved0 = 0;
    o->edge_visits = p->algo == SRT_ALGO_LEVEL ? p->lvl_visits : 0;
    o->create_device_ms = p->create_device_ms;
    return SRT_OK;
}

srt_status srt_plan_kernel_tiles(const srt_plan *p, uint64_t *tiles) {
    if (!p) return SRT_ERR_INVALID;
    if (tiles) *tiles = p->p3_tiles;
    return SRT_OK;
}

void srt_plan_destroy(srt_plan *p) {
    if (!p) return;
    hipSetDevice(p->device);
    if (p->stream) hipStreamSynchronize(p->stream);
    if (p->side_stream) hipStreamSynchronize(p->side_stream);
    if (p->comm_stream) hipStreamSynchronize(p->comm_stream);
    free_plan_buffers(p);
    (void)give_stream_set(p);  // synchronised above: reusable by the next plan
    for (hipEvent_t e : p->ev) hipEventDestroy(e);
    for (hipEvent_t e : p->ev_tail) hipEventDestroy(e);
    for (hipEvent_t e : p->cspan) hipEventDestroy(e);
    for (hipEvent_t e : {p->ev_begin, p->ev_end, p->ev_cross, p->ev_pivot, p->ev_row, p->ev_bcast, p->ev_loss0,
                         p->ev_loss1, p->ev_upload})
        if (e) hipEventDestroy(e);
    if (p->side_stream) hipStreamDestroy(p->side_stream);
    if (p->comm_stream) hipStreamDestroy(p->comm_stream);
    if (p->own_stream && p->stream) hipStreamDestroy(p->stream);
    delete p;
}

// loss-pass rows of every rank of a sharded dense build: the table rows whose
// source lies in the rank's closure block-rows (rows_per graph rows each; all
// ranks compute the same lists).  Row staging and the exchange buffers are
// sized by them and reallocated at the next run.
namespace {
srt_status build_loss_rows(srt_plan *p, int W, uint32_t rows_per, srt_err *err) {
    std::vector<std::vector<uint32_t>> lists(W);
    for (uint32_t i = 0; i < p->n; ++i) lists[std::min<uint32_t>(p->nodes[i] / rows_per, W - 1)].push_back(i);
    p->lrow_cnt.assign(W, 0);
    uint32_t most = 1;
    for (int r = 0; r < W; ++r) {
        p->lrow_cnt[r] = (uint32_t)lists[r].size();
        most = std::max(most, p->lrow_cnt[r]);
    }
    // chunks of >= 64 rows, 8 at most (each chunk's all-gather runs behind
    // the next chunk's fold and its expansion behind the next all-gather:
    // emulated C3 8 ranks 19.2 ms at 4 chunks, 18.9 at 8)
    const uint32_t q = std::max<uint32_t>(1, std::min<uint32_t>(8, most / 64));
    p->tail_q = q;
    p->tail_cr = (most + q - 1) / q;
    p->lrow_max = q * p->tail_cr;
    std::vector<uint32_t> flat((size_t)W * p->lrow_max, ~0u);
    for (int r = 0; r < W; ++r)
        for (uint32_t k = 0; k < p->lrow_cnt[r]; ++k) {
            const uint32_t c = k / p->tail_cr;
            flat[((size_t)c * W + r) * p->tail_cr + k % p->tail_cr] = lists[r][k];
        }
    while (p->ev_tail.size() < 2 * (size_t)q) {
        hipEvent_t ev;
        if (hipEventCreateWithFlags(&ev, hipEventDisableTiming) != hipSuccess) break;
        p->ev_tail.push_back(ev);
    }
    void *a = nullptr;
    hipError_t e = hipMalloc(&a, flat.size() * 4);
    if (e == hipSuccess) e = hipMemcpy(a, flat.data(), flat.size() * 4, hipMemcpyHostToDevice);
    if (e != hipSuccess) {
        hipFree(a);
        return hip_fail(err, e, "loss-pass row lists");
    }
    hipFree(p->d_lrows);
    p->d_lrows = (uint32_t *)a;
    hipFree(p->d_slat);
    hipFree(p->d_sloss);
    p->d_slat = nullptr;
    p->d_sloss = nullptr;
    if (p->h_tinfo) hipHostFree(p->h_tinfo);
    p->h_tinfo = nullptr;
    hipFree(p->d_tinfo);
    p->d_tinfo = nullptr;
    return SRT_OK;
}
}  // namespace

srt_status srt_plan_bind_comm(srt_plan *p, srt_comm *comm, srt_err *err) {
    clear_err(err);
    if (!p || !comm) {
        set_err(err, SRT_ERR_INVALID, "null plan or communicator");
        return SRT_ERR_INVALID;
    }
    HIP_TRY(hipSetDevice(p->device), "hipSetDevice");
    {
        // table rows shard with no exchange until the end (SSSP sources; the
        // dense build's loss pass): rank r owns rows [r*per, (r+1)*per) (the
        // last rank's tail past n is padding), and the table is allocated
        // with per*nranks rows for an equal-chunk all-gather
        const uint32_t W = (uint32_t)comm->nranks, per = (p->n + W - 1) / W;
        const uint32_t rows_alloc = per * W;
        if (rows_alloc > p->rows_alloc) {
            void *a = nullptr, *b = nullptr;
            hipError_t e = hipMalloc(&a, std::max<size_t>((size_t)rows_alloc * p->n, 1) * 8);
            if (e == hipSuccess) e = hipMalloc(&b, std::max<size_t>((size_t)rows_alloc * p->n, 1) * 4);
            if (e != hipSuccess) {
                hipFree(a);
                return hip_fail(err, e, "hipMalloc(table rows)");
            }
            hipFree(p->d_out_lat);
            hipFree(p->d_out_loss);
            p->d_out_lat = (uint64_t *)a;
            p->d_out_loss = (float *)b;
            p->rows_alloc = rows_alloc;
        }
        void *rs = nullptr;
        hipError_t e = hipMalloc(&rs, 2 * sizeof(unsigned long long) * W);
        if (e != hipSuccess) return hip_fail(err, e, "hipMalloc(rank stats)");
        hipFree(p->d_rstats);
        p->d_rstats = (unsigned long long *)rs;
        p->comm = comm;
        p->row0 = std::min<uint32_t>(per * (uint32_t)comm->rank, p->n);
        p->row1 = std::min<uint32_t>(p->row0 + per, p->n);
        char d[64];
        std::snprintf(d, sizeof d, " ranks=%d rows=[%u,%u)", comm->nranks, p->row0, p->row1);
        p->desc += d;
        if (p->algo == SRT_ALGO_SSSP) return SRT_OK;
        if (p->algo == SRT_ALGO_LEVEL) {
            // rows dealt by node index ranges, solved into a 6-byte staging
            // and all-gathered chunk by chunk (srt_loss.hip level_sharded)
            if (srt_status st = build_loss_rows(p, comm->nranks, (p->V + W - 1) / W, err); st != SRT_OK) return st;
            return SRT_OK;
        }
    }
    // pad the node range so every rank owns the same number of block-rows
    // (equal all-gather chunks); padded nodes are isolated and never in use
    const uint32_t unit = (uint32_t)srt::FW_B * (uint32_t)comm->nranks;
    const uint32_t Vp = std::max<uint32_t>(((p->V + unit - 1) / unit) * unit, unit);
    if (Vp != p->Vp) {
        void *ptr = nullptr;
        hipError_t e = hipMalloc(&ptr, (size_t)Vp * Vp * srt::key_bytes(p->key_type));
        if (e != hipSuccess) return hip_fail(err, e, "hipMalloc(D)");
        HIP_TRY(hipFree(p->d_D), "hipFree");
        p->d_D = (uint64_t *)ptr;
        p->Vp = Vp;
    }
    const uint32_t nblk = p->Vp / srt::FW_B, per = nblk / (uint32_t)comm->nranks;
    p->rb0 = per * (uint32_t)comm->rank;
    p->rb1 = p->rb0 + per;
    if (srt_status st = build_loss_rows(p, comm->nranks, per * srt::FW_B, err); st != SRT_OK) return st;
    char d[64];
    std::snprintf(d, sizeof d, " closure-rows=[%u,%u)", p->rb0 * srt::FW_B, p->rb1 * srt::FW_B);
    p->desc += d;
    return SRT_OK;
}

srt_status srt_plan_shard_rows(srt_plan *p, int nranks, int rank, srt_err *err) {
    clear_err(err);
    if (!p || nranks < 1 || rank < 0 || rank >= nranks) {
        set_err(err, SRT_ERR_INVALID, "null plan or rank outside [0, nranks)");
        return SRT_ERR_INVALID;
    }
    if (p->comm || p->row_shard) {
        set_err(err, SRT_ERR_INVALID, "plan already sharded");
        return SRT_ERR_INVALID;
    }
    if (p->algo != SRT_ALGO_LEVEL && p->algo != SRT_ALGO_SSSP) {
        set_err(err, SRT_ERR_UNSUPPORTED,
                "row sharding without an exchange needs independent source rows (LEVEL or SSSP plans); "
                "bind a communicator for Floyd-Warshall");
        return SRT_ERR_UNSUPPORTED;
    }
    p->row0 = (uint32_t)((uint64_t)p->n * rank / nranks);
    p->row1 = (uint32_t)((uint64_t)p->n * (rank + 1) / nranks);
    p->row_shard = true;
    // measurement only (bench.py --rank-share): this rank's share of a build
    // whose class CSR is sharded too, the all-gather modelled (level_csr_sharded)
    if (const char *e = std::getenv("SRT_LVL_SHARD_EMU"); e && std::atoi(e) == 1 && nranks > 1)
        p->lvl_emu_ranks = (uint32_t)nranks;
    char d[80];
    std::snprintf(d, sizeof d, " shard=%d/%d rows=[%u,%u)", rank, nranks, p->row0, p->row1);
    p->desc += d;
    return SRT_OK;
}

namespace {

constexpr int DEPTH_MAX = 4;
// Pieces of 8 Mi entries (64 MB), 3 in flight: C3 (16k), 4 calls each, the
// table on the host 42-44 ms after the fold starts; 2 in flight measured
// bimodal (45 or 80 ms: the DMA idles whenever the host is still expanding
// the piece whose buffer it needs next); 4 Mi or 16 Mi pieces no better.
void fetch_geometry(uint64_t *piece, int *depth) {
    *piece = 1ull << 23;
    *depth = 3;
}

// The RoutingInfo's record arrays for an n x n table (2 MB aligned, on
// transparent huge pages) touched on T host threads: the first touch of fresh
// memory (page faults + the kernel's zeroing, ~1.6 GB for C3) costs more than
// the download itself, so srt_routing_info_build runs this while the closure
// is on the GPU and the download then copies into warm pages.
bool ct_alloc(srt::CompactTable *ct, uint32_t n, uint64_t g, bool rec6, int T) {
    ct->release();
    ct->n = n;
    ct->g = g;
    ct->bytes = rec6 ? SRT_RI_REC6 : SRT_RI_REC8;
    const uint64_t nn = std::max<uint64_t>((uint64_t)n * n, 1);
    auto big = [](uint64_t bytes) -> void * {
        const uint64_t HP = 2ull << 20, b = (bytes + HP - 1) / HP * HP;
        void *q = std::aligned_alloc(HP, b);
        if (q) (void)madvise(q, b, MADV_HUGEPAGE);
        return q;
    };
    if (rec6) {
        ct->lat16 = static_cast<uint16_t *>(big(nn * 2));
        ct->loss = static_cast<float *>(big(nn * 4));
    } else {
        ct->rec8 = static_cast<uint2 *>(big(nn * 8));
    }
    if ((rec6 && (!ct->lat16 || !ct->loss)) || (!rec6 && !ct->rec8)) {
        ct->release();
        return false;
    }
    auto touch = [](void *q, uint64_t bytes, int w, int T) {
        const uint64_t a = bytes * w / T, b = bytes * (w + 1) / T;
        std::memset(static_cast<uint8_t *>(q) + a, 0, b - a);
    };
    std::vector<std::thread> pool;
    for (int w = 0; w < T; ++w)
        pool.emplace_back([&, w] {
            if (ct->lat16) touch(ct->lat16, nn * 2, w, T);
            if (ct->loss) touch(ct->loss, nn * 4, w, T);
            if (ct->rec8) touch(ct->rec8, nn * 8, w, T);
        });
    for (auto &t : pool) t.join();
    return true;
}

// End-to-end download of a kp.lat32 table in 8-byte records (latency / g as
// u32 + loss bits: half the PCIe bytes of srt_path), pipelined three ways:
// the device packs and copies piece c + 1 into one pinned buffer while host
// threads move piece c from the other into its destination, and the fold of
// later rows still runs on the main stream.  Piece c waits for the fold chunk
// holding its last entry (ev_fold).  Destination: the caller's srt_path table
// (expanded; the diagonal then rewritten from the host self-loops, which need
// not fit a record's latency field), or ct (the records kept as they are).
srt_status fetch_pipelined8(srt_plan *p, srt_path *out, srt::CompactTable *ct, uint8_t *pinned, srt_err *err) {
    Trace tr;
    const uint64_t nn = (uint64_t)p->n * p->n, per_fold = (uint64_t)p->fold_chunk_rows * p->n;
    uint64_t PIECE;
    int DEPTH;
    fetch_geometry(&PIECE, &DEPTH);
    // u16-key plans (every finite latency < 0x4000 units): 6-byte records, a
    // piece = its u16 latencies, then (16-byte aligned) its f32 losses
    const bool rec6 = p->key_type == srt::KEY_U16 && !std::getenv("SRT_FETCH8");
    // every finite latency <= 510 units (the key proof's bound): 5 bytes over
    // PCIe instead of 6 (C3: 1.34 GB instead of 1.61), expanded on the host
    // into the same 6-byte arrays (SRT_FETCH6=1 keeps the 6-byte transfer)
    const bool rec5 = rec6 && p->kp.lmax <= 510 && !std::getenv("SRT_FETCH6");
    auto loss_off = [rec5](uint64_t cnt) { return ((rec5 ? cnt : cnt * 2) + 15) & ~15ull; };
    const uint32_t np = (uint32_t)((nn + PIECE - 1) / PIECE);
    // the record arrays: prepared (and touched) while the closure ran, else now
    if (ct && !(ct->n == p->n && ct->bytes == (rec6 ? SRT_RI_REC6 : SRT_RI_REC8) && (rec6 ? ct->lat16 != nullptr : ct->rec8 != nullptr)) &&
        !ct_alloc(ct, p->n, p->kp.g, rec6, host_threads(nn))) {
        set_err(err, SRT_ERR_OOM, "out of host memory (routing table)");
        return SRT_ERR_OOM;
    }
    if (!p->d_pack8) HIP_TRY(hipMalloc(&p->d_pack8, PIECE * 8 * DEPTH), "hipMalloc(pack8)");
    uint2 *h[DEPTH_MAX];
    hipEvent_t ev[DEPTH_MAX];
    for (int i = 0; i < DEPTH; ++i) {
        h[i] = reinterpret_cast<uint2 *>(pinned) + (uint64_t)i * PIECE;
        HIP_TRY(hipEventCreateWithFlags(&ev[i], hipEventDisableTiming), "event");
    }
    hipStream_t C = p->comm_stream;
    auto enqueue = [&](uint32_t c) -> hipError_t {
        const uint64_t first = (uint64_t)c * PIECE, cnt = std::min(PIECE, nn - first);
        hipError_t e = hipStreamWaitEvent(C, p->ev_fold[(first + cnt - 1) / per_fold], 0);
        if (e != hipSuccess) return e;
        uint2 *dst = reinterpret_cast<uint2 *>(p->d_pack8) + (uint64_t)(c % DEPTH) * PIECE;
        if (rec5) {
            srt::pack_paths5(p, first, cnt, dst, loss_off(cnt), C);
            e = hipMemcpyAsync(h[c % DEPTH], dst, loss_off(cnt) + cnt * 4, hipMemcpyDeviceToHost, C);
        } else if (rec6) {
            srt::pack_paths6(p, first, cnt, dst, loss_off(cnt), C);
            e = hipMemcpyAsync(h[c % DEPTH], dst, loss_off(cnt) + cnt * 4, hipMemcpyDeviceToHost, C);
        } else {
            srt::pack_paths8(p, first, cnt, dst, C);
            e = hipMemcpyAsync(h[c % DEPTH], dst, cnt * 8, hipMemcpyDeviceToHost, C);
        }
        return e == hipSuccess ? hipEventRecord(ev[c % DEPTH], C) : e;
    };
    const uint64_t g = p->kp.g;
    const int T = host_threads(nn);
    // expansion of entries [a, b) of piece c into the caller's table: one
    // 16-byte non-temporal store per entry when the table is 16-byte aligned
    // (no read-for-ownership of the destination lines)
    const bool nt = out && (reinterpret_cast<uintptr_t>(out) & 15) == 0;
    auto expand_range = [&](uint32_t c, uint64_t a, uint64_t b) {
        const uint64_t first = (uint64_t)c * PIECE;
        const uint2 *src = h[c % DEPTH];
        if (ct) {  // the records as they are
            if (b <= a) return;
            if (rec5) {  // 9-bit units (511: unreachable) into the u16 array, the loss bits into theirs
                const uint64_t cnt = std::min(PIECE, nn - first);
                const uint8_t *l8 = reinterpret_cast<const uint8_t *>(src);
                const uint32_t *lw = reinterpret_cast<const uint32_t *>(reinterpret_cast<const uint8_t *>(src) + loss_off(cnt));
                uint16_t *dl = ct->lat16 + first;
                uint32_t *dp = reinterpret_cast<uint32_t *>(ct->loss + first);
                for (uint64_t i = a; i < b; ++i) {
                    const uint32_t w = lw[i], u = l8[i] | ((w >> 31) << 8);
                    dl[i] = u == 511u ? (uint16_t)0xffffu : (uint16_t)u;
                    dp[i] = w & 0x7fffffffu;
                }
            } else if (rec6) {
                const uint64_t cnt = std::min(PIECE, nn - first);
                std::memcpy(ct->lat16 + first + a, reinterpret_cast<const uint16_t *>(src) + a, (b - a) * 2);
                std::memcpy(ct->loss + first + a,
                            reinterpret_cast<const float *>(reinterpret_cast<const uint8_t *>(src) + loss_off(cnt)) + a,
                            (b - a) * 4);
            } else {
                std::memcpy(ct->rec8 + first + a, src + a, (b - a) * 8);
            }
            return;
        }
        srt_path *dst = out + first;
        if (rec5) {
            const uint64_t cnt = std::min(PIECE, nn - first);
            const uint8_t *l8 = reinterpret_cast<const uint8_t *>(src);
            const uint32_t *lw = reinterpret_cast<const uint32_t *>(reinterpret_cast<const uint8_t *>(src) + loss_off(cnt));
            for (uint64_t i = a; i < b; ++i) {
                const uint32_t w = lw[i], u = l8[i] | ((w >> 31) << 8);
                const uint64_t l = u == 511u ? ~0ull : (uint64_t)u * g;
                if (nt) {
                    _mm_stream_si128(reinterpret_cast<__m128i *>(dst + i),
                                     _mm_set_epi64x((long long)(w & 0x7fffffffu), (long long)l));
                } else {
                    srt_path q;
                    q.latency_ns = l;
                    const uint32_t lb = w & 0x7fffffffu;
                    std::memcpy(&q.packet_loss, &lb, 4);
                    q._pad = 0;
                    dst[i] = q;
                }
            }
        } else if (rec6) {
            const uint64_t cnt = std::min(PIECE, nn - first);
            const uint16_t *l16 = reinterpret_cast<const uint16_t *>(src);
            const uint32_t *lb = reinterpret_cast<const uint32_t *>(reinterpret_cast<const uint8_t *>(src) + loss_off(cnt));
            for (uint64_t i = a; i < b; ++i) {
                const uint64_t l = l16[i] == 0xffffu ? ~0ull : (uint64_t)l16[i] * g;
                if (nt) {
                    _mm_stream_si128(reinterpret_cast<__m128i *>(dst + i), _mm_set_epi64x((long long)lb[i], (long long)l));
                } else {
                    srt_path q;
                    q.latency_ns = l;
                    std::memcpy(&q.packet_loss, lb + i, 4);
                    q._pad = 0;
                    dst[i] = q;
                }
            }
        } else if (nt) {
            for (uint64_t i = a; i < b; ++i) {
                const uint2 r = src[i];
                const uint64_t l = r.x == 0xffffffffu ? ~0ull : (uint64_t)r.x * g;
                _mm_stream_si128(reinterpret_cast<__m128i *>(dst + i), _mm_set_epi64x((long long)r.y, (long long)l));
            }
        } else {
            for (uint64_t i = a; i < b; ++i) {
                const uint2 r = src[i];
                srt_path q;
                q.latency_ns = r.x == 0xffffffffu ? ~0ull : (uint64_t)r.x * g;
                std::memcpy(&q.packet_loss, &r.y, 4);
                q._pad = 0;
                dst[i] = q;
            }
        }
    };
    std::atomic<int> ready{-1}, stop{0};
    std::atomic<uint64_t> done{0};
    auto expand = [&](int w) {
        for (uint32_t c = 0; c < np; ++c) {
            while (ready.load(std::memory_order_acquire) < (int)c) {
                if (stop.load(std::memory_order_relaxed)) return;
                std::this_thread::yield();
            }
            const uint64_t first = (uint64_t)c * PIECE, cnt = std::min(PIECE, nn - first);
            expand_range(c, cnt * w / T, cnt * (w + 1) / T);
            _mm_sfence();
            done.fetch_add(1, std::memory_order_acq_rel);
        }
    };
    hipError_t e = hipSuccess;
    for (uint32_t c = 0; c < (uint32_t)DEPTH && c < np && e == hipSuccess; ++c) e = enqueue(c);
    std::vector<std::thread> pool;
    for (int w = 1; w < T && e == hipSuccess; ++w) pool.emplace_back(expand, w);
    double wait_dma = 0.0, wait_expand = 0.0;  // SRT_TRACE: where the main thread waited
    for (uint32_t c = 0; c < np && e == hipSuccess; ++c) {
        auto t0 = std::chrono::steady_clock::now();
        e = hipEventSynchronize(ev[c % DEPTH]);
        if (e != hipSuccess) break;
        auto t1 = std::chrono::steady_clock::now();
        if (c > 0) wait_dma += std::chrono::duration<double, std::milli>(t1 - t0).count();
        if (c == 0) tr.mark("fetch8: first piece on the host");
        ready.store((int)c, std::memory_order_release);
        // this thread expands its own slice, then waits for the others
        expand_range(c, 0, std::min(PIECE, nn - (uint64_t)c * PIECE) / T);
        _mm_sfence();
        while (done.load(std::memory_order_acquire) < (uint64_t)(c + 1) * (T - 1)) std::this_thread::yield();
        wait_expand += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t1).count();
        if (c + DEPTH < np) e = enqueue(c + DEPTH);
    }
    stop.store(1);
    for (auto &th : pool) th.join();
    if (tr.on)
        std::fprintf(stderr, "[srt] fetch8: %u pieces of %d-byte records, %d threads, nt=%d, %s: waited %.1f ms on DMA, "
                     "%.1f ms expanding\n", np, rec5 ? 5 : rec6 ? 6 : 8, T, (int)nt, ct ? "kept" : "expanded", wait_dma,
                     wait_expand);
    tr.mark("fetch8: pieces downloaded + expanded");
    for (int i = 0; i < DEPTH; ++i) (void)hipEventDestroy(ev[i]);
    if (e != hipSuccess) return hip_fail(err, e, "compact download");
    // the diagonal: the raw self-loops (mod.rs:210-217), from the host
    if (ct) {
        ct->diag.resize(p->n);
        for (uint32_t i = 0; i < p->n; ++i) ct->diag[i] = srt_path{p->h_sl_lat[i], p->h_sl_loss[i], 0u};
    } else {
        for (uint32_t i = 0; i < p->n; ++i) out[(uint64_t)i * p->n + i] = srt_path{p->h_sl_lat[i], p->h_sl_loss[i], 0u};
    }
    return SRT_OK;
}

// End-to-end download behind the chunked fold (fw_loss with fold_chunk_rows):
// chunk c's rows are packed and copied to the host on the comm stream (idle
// on one GPU) once ev_fold[c] fires, while the fold of chunk c + 1 runs.
// ct: keep compact records (kp.lat32 plans) -- else ct gets an srt_path table.
srt_status fetch_pipelined(srt_plan *p, srt_path *out, srt::CompactTable *ct, uint64_t *min_latency_ns,
                           srt_err *err) {
    const uint64_t nn = (uint64_t)p->n * p->n, per = (uint64_t)p->fold_chunk_rows * p->n;
    const uint32_t nc = (uint32_t)((nn + per - 1) / per);
    if (!p->d_pack) {
        void *ptr = nullptr;
        hipError_t e = hipMalloc(&ptr, per * sizeof(srt_path));
        if (e != hipSuccess) return hip_fail(err, e, "hipMalloc(pack)");
        p->d_pack = (srt_path *)ptr;
    }
    hipStream_t C = p->comm_stream;
    // compact (8-byte) records when every latency fits u32 units (knob
    // SRT_FETCH16=1: the 16-byte srt_path download, for A/B)
    if (p->kp.lat32 && !std::getenv("SRT_FETCH16")) {
        PinnedPool &pp = g_pinned;
        std::unique_lock<std::mutex> lk(pp.m, std::try_to_lock);
        if (lk.owns_lock()) {
            uint64_t piece;
            int depth;
            fetch_geometry(&piece, &depth);
            if (pp.ensure(std::max<size_t>(PINNED_BYTES, (size_t)depth * piece * 8))) {
                srt_status s = fetch_pipelined8(p, out, ct, reinterpret_cast<uint8_t *>(pp.buf), err);
                if (s == SRT_OK) s = srt_plan_sync(p, err);
                if (s == SRT_OK) s = srt_plan_fetch(p, nullptr, min_latency_ns, err);
                return s;
            }
        }
    }
    if (ct) {
        ct->release();
        ct->n = p->n;
        ct->bytes = SRT_RI_PATH16;
        ct->full = static_cast<srt_path *>(std::malloc(std::max<uint64_t>(nn, 1) * sizeof(srt_path)));
        if (!ct->full) {
            set_err(err, SRT_ERR_OOM, "out of host memory (routing table)");
            return SRT_ERR_OOM;
        }
        out = ct->full;
    }
    for (uint32_t c = 0; c < nc; ++c) {
        const uint64_t first = (uint64_t)c * per, cnt = std::min(per, nn - first);
        HIP_TRY(hipStreamWaitEvent(C, p->ev_fold[c], 0), "wait fold chunk");
        srt::pack_paths(p, first, cnt, p->d_pack, C);
        HIP_TRY(hipMemcpyAsync(out + first, p->d_pack, cnt * sizeof(srt_path), hipMemcpyDeviceToHost, C),
                "download");
    }
    HIP_TRY(hipStreamSynchronize(C), "sync");
    srt_status s = srt_plan_sync(p, err);
    // connectivity (the reference's assert) and the min latency; the table is home
    if (s == SRT_OK) s = srt_plan_fetch(p, nullptr, min_latency_ns, err);
    if (s == SRT_OK && ct) {
        ct->diag.resize(p->n);
        for (uint32_t i = 0; i < p->n; ++i) ct->diag[i] = out[(uint64_t)i * p->n + i];
    }
    return s;
}

// The in-process multi-GPU build of a level plan (srt_opts.n_gpus > 1, the
// family AUTO picks for C1-C3): rank 0's plan did the one CSR scan and
// upload; its class CSRs (the whole input of a solve: ~0.1 GB at C3) go to
// every other device over xGMI (hipMemcpyPeerAsync; ranks on the same device
// share them), every rank solves its contiguous rows into a 6-byte staging
// (u16 latency units + f32 loss) and downloads them over its own PCIe link
// straight into the caller's records (RoutingInfo) or, expanded by its
// thread, into the caller's srt_path rows.  No table exchange between the
// GPUs: Shadow's one consumer is the host (sim_config.rs:136-140, 424-461).
// SRT_MULTI_EMULATE=1 (measurement only): rank 0's share alone -- its rows,
// the others skipped (their rows are left unwritten).
srt_status build_multi_level(srt_plan *p0, const std::vector<int32_t> &devs, srt_path *out, srt::CompactTable *ct,
                             uint64_t *min_latency_ns, srt_err *err) {
    Trace tr;
    const int N = (int)devs.size();
    const uint32_t n = p0->n;
    const bool emulate = std::getenv("SRT_MULTI_EMULATE") && std::atoi(std::getenv("SRT_MULTI_EMULATE")) != 0;
    HIP_TRY(hipSetDevice(p0->device), "hipSetDevice");
    if (srt_status s = upload_deferred_loss(p0, err); s != SRT_OK) return s;
    if (srt_status s = srt::level_prepare(p0, err); s != SRT_OK) return s;
    hipEvent_t ready = nullptr;
    HIP_TRY(hipEventCreateWithFlags(&ready, hipEventDisableTiming), "event");
    HIP_TRY(hipEventRecord(ready, p0->stream), "event record");
    tr.mark("multi: class CSRs on rank 0");
    // quantized plans (latency units past u16): u32 staging, 8-byte records
    const bool quant = p0->lvl_q != 0;
    if (ct) {
        const int T = host_threads((uint64_t)n * n);
        if (!ct_alloc(ct, n, p0->kp.g, !quant, T)) {
            (void)hipEventDestroy(ready);
            set_err(err, SRT_ERR_OOM, "out of host memory (routing table)");
            return SRT_ERR_OOM;
        }
    }
    const srt::LevelCtx c0 = srt::level_ctx(p0);
    const uint64_t vc1 = (uint64_t)p0->V * p0->t_cls + 1, ents = p0->lvl_cap + 1024;
    // the copies of the solve's inputs on the other devices are checked against
    // rank 0's originals (srt::checksum; SRT_ERR_COMM on a mismatch).  Knobs
    // (tests on one GPU): SRT_MULTI_FORCE_COPY=1 copies to ranks that share
    // rank 0's device too; SRT_TEST_CORRUPT_PEER=r flips a byte of rank r's copy
    const bool force_copy = std::getenv("SRT_MULTI_FORCE_COPY") && std::atoi(std::getenv("SRT_MULTI_FORCE_COPY")) == 1;
    const int corrupt_rank = std::getenv("SRT_TEST_CORRUPT_PEER") ? std::atoi(std::getenv("SRT_TEST_CORRUPT_PEER")) : -1;
    struct CopySrc {
        const void *p;
        uint64_t bytes;
    };
    const bool alias0 = c0.ce_in == c0.ce_out;
    const CopySrc srcs[6] = {{c0.tcls, 2 * vc1 * 4}, {c0.ce_out, ents * 8}, {alias0 ? nullptr : c0.ce_in, ents * 8},
                             {c0.nodes, (uint64_t)n * 4}, {c0.sl_lat, (uint64_t)n * 8}, {c0.sl_loss, (uint64_t)n * 4}};
    unsigned long long h_ck0[6] = {};
    bool any_copy = false;
    for (int r = 1; r < N; ++r) any_copy |= devs[r] != devs[0] || force_copy;
    if (any_copy && !emulate) {
        unsigned long long *d_ck = nullptr;
        hipError_t e = hipMalloc(&d_ck, sizeof h_ck0);
        for (int k = 0; k < 6 && e == hipSuccess; ++k)
            if (srcs[k].p) srt::checksum(srcs[k].p, srcs[k].bytes, d_ck + k, p0->stream);
        if (e == hipSuccess) e = hipMemcpyAsync(h_ck0, d_ck, sizeof h_ck0, hipMemcpyDeviceToHost, p0->stream);
        if (e == hipSuccess) e = hipStreamSynchronize(p0->stream);
        (void)hipFree(d_ck);
        if (e != hipSuccess) {
            (void)hipEventDestroy(ready);
            return hip_fail(err, e, "class CSR checksums");
        }
    }
    std::vector<srt_status> sts(N, SRT_OK);
    std::vector<srt_err> errs(N);
    std::vector<unsigned long long> mins(N, ~0ull), unre(N, 0);
    auto rank_fn = [&](int r) {
        srt_err *e2 = &errs[r];
        std::memset(e2, 0, sizeof *e2);
        const uint32_t r0 = (uint32_t)((uint64_t)n * r / N), r1 = (uint32_t)((uint64_t)n * (r + 1) / N);
        const uint64_t rows = r1 - r0;
        std::vector<void *> owned;
        hipStream_t st = nullptr;
        auto fail = [&](hipError_t e, const char *what) {
            sts[r] = hip_fail(e2, e, what);
        };
        auto dev_alloc = [&](size_t bytes) -> void * {
            void *q = nullptr;
            if (hipMalloc(&q, std::max<size_t>(bytes, 1)) != hipSuccess) return nullptr;
            owned.push_back(q);
            return q;
        };
        hipError_t e = hipSetDevice(devs[r]);
        srt::LevelCtx c = c0;
        c.device = devs[r];
        c.visits = nullptr;
        c.row_ctr = nullptr;  // ranks solve concurrently: rows dealt statically
        if (e == hipSuccess) e = r == 0 ? hipSuccess : hipStreamCreateWithFlags(&st, hipStreamNonBlocking);
        if (r == 0) st = p0->stream;
        c.stream = st;
        if (e == hipSuccess) e = hipStreamWaitEvent(st, ready, 0);
        bool corrupt = false;
        if (e == hipSuccess && (devs[r] != devs[0] || (force_copy && r != 0))) {
            // the solve's inputs from rank 0's device
            uint32_t *tcls = (uint32_t *)dev_alloc(2 * vc1 * 4);
            const bool alias = c0.ce_in == c0.ce_out;  // symmetric plan: one entry array
            uint64_t *eo = (uint64_t *)dev_alloc(ents * 8), *ei = alias ? eo : (uint64_t *)dev_alloc(ents * 8);
            uint32_t *nd = (uint32_t *)dev_alloc((size_t)n * 4);
            uint64_t *sl = (uint64_t *)dev_alloc((size_t)n * 8);
            float *sp = (float *)dev_alloc((size_t)n * 4);
            if (!tcls || !eo || !ei || !nd || !sl || !sp) e = hipErrorOutOfMemory;
            if (e == hipSuccess) e = hipMemcpyPeerAsync(tcls, devs[r], c0.tcls, devs[0], 2 * vc1 * 4, st);
            if (e == hipSuccess) e = hipMemcpyPeerAsync(eo, devs[r], c0.ce_out, devs[0], ents * 8, st);
            if (e == hipSuccess && !alias) e = hipMemcpyPeerAsync(ei, devs[r], c0.ce_in, devs[0], ents * 8, st);
            if (e == hipSuccess) e = hipMemcpyPeerAsync(nd, devs[r], c0.nodes, devs[0], (size_t)n * 4, st);
            if (e == hipSuccess) e = hipMemcpyPeerAsync(sl, devs[r], c0.sl_lat, devs[0], (size_t)n * 8, st);
            if (e == hipSuccess) e = hipMemcpyPeerAsync(sp, devs[r], c0.sl_loss, devs[0], (size_t)n * 4, st);
            c.tcls = tcls;
            c.ce_out = eo;
            c.ce_in = ei;
            c.nodes = nd;
            c.sl_lat = sl;
            c.sl_loss = sp;
            // every copy against rank 0's checksum before anything reads it
            unsigned long long *d_ck = (unsigned long long *)dev_alloc(6 * 8);
            if (!d_ck) e = hipErrorOutOfMemory;
            if (e == hipSuccess && r == corrupt_rank) srt::corrupt_byte(sp, (uint64_t)n * 4, st);  // a loss value
            const void *dsts[6] = {tcls, eo, alias ? nullptr : ei, nd, sl, sp};
            unsigned long long h_ck[6] = {};
            for (int k = 0; k < 6 && e == hipSuccess; ++k)
                if (srcs[k].p) srt::checksum(dsts[k], srcs[k].bytes, d_ck + k, st);
            if (e == hipSuccess) e = hipMemcpyAsync(h_ck, d_ck, sizeof h_ck, hipMemcpyDeviceToHost, st);
            if (e == hipSuccess) e = hipStreamSynchronize(st);
            for (int k = 0; k < 6 && e == hipSuccess; ++k) corrupt |= srcs[k].p && h_ck[k] != h_ck0[k];
        }
        if (corrupt) {
            if (st && r != 0) (void)hipStreamSynchronize(st);
            for (void *q : owned) (void)hipFree(q);
            if (st && r != 0) (void)hipStreamDestroy(st);
            set_err(e2, SRT_ERR_COMM, "multi-GPU level build: a device's copy of the class CSRs differs from rank 0's "
                                      "(checksum)");
            sts[r] = SRT_ERR_COMM;
            return;
        }
        // staging: u16 (u32 when quantized) latency units + f32 loss, or --
        // quantized into a RoutingInfo -- its 8-byte records as they are
        const size_t lw = quant ? 4 : 2;
        const uint32_t mode = quant ? (ct ? 3u : 2u) : 1u;
        void *s16 = nullptr;
        float *sloss = nullptr;
        unsigned long long *dst = nullptr;
        if (e == hipSuccess) {
            s16 = dev_alloc(mode == 3 ? rows * n * 8 : rows * n * lw + 256);
            sloss = mode == 3 ? nullptr : (float *)dev_alloc(rows * n * 4);
            dst = (unsigned long long *)dev_alloc(4 * 8);
            // the quantized solve's per-workgroup scratch: every rank its own
            // (ranks sharing a device run concurrently)
            if (quant) c.lmem = (uint16_t *)dev_alloc(srt::level_scratch_bytes(devs[r], p0->V, true));
            if (!s16 || (mode != 3 && !sloss) || !dst || (quant && !c.lmem)) e = hipErrorOutOfMemory;
        }
        if (e == hipSuccess && rows) {
            srt::level_stats_init(dst, st);
            srt::level_solve_stage(c, r0, r1, (uint32_t)p0->kp.lmax, s16, sloss, mode, dst);
        }
        unsigned long long hs[2] = {~0ull, 0};
        std::vector<uint8_t> h16;
        std::vector<float> hl;
        if (e == hipSuccess && rows) {
            if (ct && mode == 3) {
                // straight into the RoutingInfo's 8-byte records
                e = hipMemcpyAsync(ct->rec8 + (uint64_t)r0 * n, s16, rows * n * 8, hipMemcpyDeviceToHost, st);
            } else if (ct) {
                // straight into the RoutingInfo's 6-byte records
                e = hipMemcpyAsync(ct->lat16 + (uint64_t)r0 * n, s16, rows * n * 2, hipMemcpyDeviceToHost, st);
                if (e == hipSuccess)
                    e = hipMemcpyAsync(ct->loss + (uint64_t)r0 * n, sloss, rows * n * 4, hipMemcpyDeviceToHost, st);
            } else {
                h16.resize(rows * n * lw);
                hl.resize(rows * n);
                e = hipMemcpyAsync(h16.data(), s16, rows * n * lw, hipMemcpyDeviceToHost, st);
                if (e == hipSuccess) e = hipMemcpyAsync(hl.data(), sloss, rows * n * 4, hipMemcpyDeviceToHost, st);
            }
            if (e == hipSuccess) e = hipMemcpyAsync(hs, dst, sizeof hs, hipMemcpyDeviceToHost, st);
            if (e == hipSuccess) e = hipStreamSynchronize(st);
        }
        if (e == hipSuccess && out && rows) {
            // expanded into the caller's srt_path rows by this rank's share of the host threads
            const uint64_t g = p0->kp.g, cnt = rows * n;
            const int T = std::max(1, host_threads(cnt) / (emulate ? 1 : N));
            const uint16_t *l16 = reinterpret_cast<const uint16_t *>(h16.data());
            const uint32_t *l32 = reinterpret_cast<const uint32_t *>(h16.data());
            auto part = [&](int w) {
                for (uint64_t k = cnt * w / T; k < cnt * (w + 1) / T; ++k) {
                    srt_path q;
                    if (quant)
                        q.latency_ns = l32[k] == ~0u ? ~0ull : (uint64_t)l32[k] * g;
                    else
                        q.latency_ns = l16[k] == 0xffffu ? ~0ull : (uint64_t)l16[k] * g;
                    q.packet_loss = hl[k];
                    q._pad = 0;
                    out[(uint64_t)r0 * n + k] = q;
                }
            };
            std::vector<std::thread> pool;
            for (int w = 1; w < T; ++w) pool.emplace_back(part, w);
            part(0);
            for (auto &t : pool) t.join();
        }
        if (st && r != 0) (void)hipStreamSynchronize(st);
        for (void *q : owned) (void)hipFree(q);
        if (st && r != 0) (void)hipStreamDestroy(st);
        if (e != hipSuccess) fail(e, "multi-GPU level solve");
        mins[r] = hs[0];
        unre[r] = hs[1];
    };
    std::vector<std::thread> th;
    for (int r = 0; r < N; ++r) {
        if (emulate && r > 0) continue;
        th.emplace_back(rank_fn, r);
    }
    for (auto &t : th) t.join();
    (void)hipSetDevice(p0->device);
    (void)hipEventDestroy(ready);
    tr.mark("multi: ranks solved + downloaded");
    for (int r = 0; r < N; ++r)
        if (sts[r] != SRT_OK) {
            if (err) *err = errs[r];
            return sts[r];
        }
    unsigned long long mn = ~0ull, un = 0;
    for (int r = 0; r < N; ++r) {
        mn = std::min(mn, mins[r]);
        un += unre[r];
    }
    if (un != 0 && !emulate) {
        char buf[200];
        const unsigned long long nn = (unsigned long long)n * n;
        std::snprintf(buf, sizeof buf, "assertion `left == right` failed\n  left: %llu\n right: %llu", nn - un, nn);
        set_err(err, SRT_ERR_DISCONNECTED, buf);
        return SRT_ERR_DISCONNECTED;
    }
    if (min_latency_ns) *min_latency_ns = mn;
    // the diagonal: the raw self-loops (mod.rs:210-217), from the host
    if (ct) {
        ct->diag.resize(n);
        for (uint32_t i = 0; i < n; ++i) ct->diag[i] = srt_path{p0->h_sl_lat[i], p0->h_sl_loss[i], 0u};
    } else {
        for (uint32_t i = 0; i < n; ++i) out[(uint64_t)i * n + i] = srt_path{p0->h_sl_lat[i], p0->h_sl_loss[i], 0u};
    }
    return SRT_OK;
}

// The multi-GPU build inside the caller's process (srt_opts.n_gpus > 1): one
// host thread and one plan per device, bound to an in-process communicator
// (srt_comm_init_local), every sharded schedule unchanged; rank 0's plan holds
// the whole table after the row all-gather and is the one fetched.  This is
// how Shadow's single process -- generate_routing_info runs once, on its main
// thread (sim_config.rs:136-140, 424-461) -- reaches every GPU of the node.
srt_status build_multi(const srt_csr *g, const uint32_t *nodes, uint32_t n, srt_path *out, srt::CompactTable *ct,
                       uint64_t *min_latency_ns, const srt_opts *opts, srt_err *err) {
    const int N = (int)opts->n_gpus;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev < 1) {
        set_err(err, SRT_ERR_HIP, "no HIP device");
        return SRT_ERR_HIP;
    }
    const bool same = (opts->flags & SRT_OPT_SAME_DEVICE) != 0;
    int first = opts->device;
    if (first < 0 && hipGetDevice(&first) != hipSuccess) first = 0;
    if (N > srt::MAX_LOCAL_RANKS || (!same && (N > ndev || first + N > ndev))) {
        set_err(err, SRT_ERR_INVALID, "srt_opts.n_gpus exceeds the visible devices (or 16)");
        return SRT_ERR_INVALID;
    }
    std::vector<int32_t> devs(N);
    for (int r = 0; r < N; ++r) devs[r] = same ? first : first + r;
    srt_plan *p0 = nullptr;
    {
        // rank 0's plan: the one CSR scan + upload and the family choice; a
        // level plan needs no other plan (build_multi_level), a closure plan
        // is rank 0's plan of the sharded run below
        srt_opts o0 = *opts;
        o0.device = devs[0];
        o0.n_gpus = 1;
        o0.flags &= ~(uint32_t)SRT_OPT_SAME_DEVICE;
        if (srt_status s = plan_create_impl(g, nodes, n, &o0, &p0, err, true); s != SRT_OK) return s;
        if (p0->algo == SRT_ALGO_LEVEL) {
            srt_status s = build_multi_level(p0, devs, out, ct, min_latency_ns, err);
            // the device's loss range check: a parse-time error, so it wins
            join_loss_check(p0);
            if (p0->h_lossbad && s != SRT_ERR_HIP) {
                (void)hipSetDevice(p0->device);
                (void)hipStreamSynchronize(p0->comm_stream);
                if (*p0->h_lossbad != ~0ull) {
                    s = SRT_ERR_INVALID;
                    set_err(err, SRT_ERR_INVALID, "Edge 'packet_loss' is not in the range [0,1]");
                }
            }
            reap_async(p0);
            return s;
        }
    }
    std::vector<srt_comm *> comms(N, nullptr);
    if (srt_status s = srt_comm_init_local(N, devs.data(), comms.data(), err); s != SRT_OK) {
        join_loss_check(p0);
        srt_plan_destroy(p0);
        return s;
    }
    std::vector<srt_plan *> plans(N, nullptr);
    plans[0] = p0;  // its losses upload in its run (run_tail), g stays valid until then
    std::vector<srt_status> sts(N, SRT_OK);
    std::vector<srt_err> errs(N);
    std::vector<std::thread> th;
    for (int r = 0; r < N; ++r)
        th.emplace_back([&, r] {
            srt_opts o = *opts;
            o.device = devs[r];
            o.n_gpus = 1;
            o.flags &= ~(uint32_t)SRT_OPT_SAME_DEVICE;
            std::memset(&errs[r], 0, sizeof errs[r]);
            srt_status s = r == 0 ? SRT_OK : plan_create_impl(g, nodes, n, &o, &plans[r], &errs[r], false);
            if (s == SRT_OK) s = srt_plan_bind_comm(plans[r], comms[r], &errs[r]);
            if (s == SRT_OK) s = srt_plan_run(plans[r], &errs[r]);
            if (s != SRT_OK) srt_comm_abort(comms[r]);  // releases the others' collectives
            sts[r] = s;
        });
    for (auto &t : th) t.join();
    // the first rank's own failure (graph errors are found by every rank
    // alike); a rank released by another's abort reports SRT_ERR_COMM
    srt_status s = SRT_OK;
    for (int r = 0; r < N && s == SRT_OK; ++r)
        if (sts[r] != SRT_OK && sts[r] != SRT_ERR_COMM) {
            s = sts[r];
            if (err) *err = errs[r];
        }
    for (int r = 0; r < N && s == SRT_OK; ++r)
        if (sts[r] != SRT_OK) {
            s = sts[r];
            if (err) *err = errs[r];
        }
    if (s == SRT_OK && ct) {
        ct->release();
        ct->n = n;
        ct->bytes = SRT_RI_PATH16;
        ct->full = static_cast<srt_path *>(std::malloc(std::max<uint64_t>((uint64_t)n * n, 1) * sizeof(srt_path)));
        if (!ct->full) {
            s = SRT_ERR_OOM;
            set_err(err, SRT_ERR_OOM, "out of host memory (routing table)");
        }
        out = ct->full;
    }
    if (s == SRT_OK) s = srt_plan_fetch(plans[0], out, min_latency_ns, err);
    if (s == SRT_OK && ct) {
        ct->diag.resize(n);
        for (uint32_t i = 0; i < n; ++i) ct->diag[i] = out[(uint64_t)i * n + i];
    }
    // rank 0's device loss range check (its deferred upload): a parse-time
    // error, so it wins over any error of the build itself
    join_loss_check(p0);
    if (p0->h_lossbad && s != SRT_ERR_HIP) {
        (void)hipSetDevice(p0->device);
        (void)hipStreamSynchronize(p0->stream);
        (void)hipStreamSynchronize(p0->comm_stream);
        if (*p0->h_lossbad != ~0ull) {
            s = SRT_ERR_INVALID;
            set_err(err, SRT_ERR_INVALID, "Edge 'packet_loss' is not in the range [0,1]");
        }
    }
    for (int r = 0; r < N; ++r) srt_plan_destroy(plans[r]);
    for (int r = 0; r < N; ++r) srt_comm_destroy(comms[r]);
    return s;
}

// srt_compute_shortest_paths' end-to-end build into `out` (srt_path) or `ct`
srt_status build_e2e(const srt_csr *g, const uint32_t *nodes, uint32_t n, srt_path *out, srt::CompactTable *ct,
                     uint64_t *min_latency_ns, const srt_opts *opts, srt_err *err) {
    srt::init_wait();
    if (opts && opts->n_gpus > 1) return build_multi(g, nodes, n, out, ct, min_latency_ns, opts, err);
    srt_plan *p = nullptr;
    Trace tr;
    srt_status s = plan_create_impl(g, nodes, n, opts, &p, err, true);
    tr.mark("e2e: create");
    if (s != SRT_OK) return s;
    // one-GPU dense build with a table wanted: the fold runs in chunks of <= 64
    // Mi entries whose downloads overlap the next chunk's fold
    const bool pipe = (out || ct) && p->n && (p->algo == SRT_ALGO_FW || p->algo == SRT_ALGO_LEVEL) && !p->comm &&
                      p->emulate_ranks <= 1;
    if (pipe)
        p->fold_chunk_rows = (uint32_t)std::max<uint64_t>(
            1, std::min<uint64_t>((uint64_t)p->n * p->n, 1ull << 26) / p->n);
    s = run_closure(p, err);
    tr.mark("e2e: closure enqueued");
    // the pinned staging of the compact download, pinned while the closure
    // runs (first call of the process without srt_init: ~1 ms per MB, too
    // slow to pay inline)
    std::thread pinner, prefault;
    if (s == SRT_OK && pipe && p->kp.lat32 && g_pinned.bytes < PINNED_BYTES)
        pinner = std::thread([] {
            std::lock_guard<std::mutex> lk(g_pinned.m);
            (void)g_pinned.ensure(PINNED_BYTES);
        });
    // RoutingInfo records: allocated and touched while the closure runs
    if (s == SRT_OK && pipe && ct && p->kp.lat32 && !std::getenv("SRT_FETCH16")) {
        const bool rec6 = p->key_type == srt::KEY_U16 && !std::getenv("SRT_FETCH8");
        const int T = host_threads((uint64_t)p->n * p->n);
        prefault = std::thread([ct, p, rec6, T] { (void)ct_alloc(ct, p->n, p->kp.g, rec6, T); });
    }
    if (s == SRT_OK) s = run_tail(p, err);  // the deferred loss upload overlaps the closure
    tr.mark("e2e: loss upload + tail enqueued");
    if (pinner.joinable()) pinner.join();
    tr.mark("e2e: pinned staging ready");
    if (prefault.joinable()) prefault.join();
    tr.mark("e2e: routing records touched");
    if (s == SRT_OK && pipe) {
        s = fetch_pipelined(p, out, ct, min_latency_ns, err);
    } else if (s == SRT_OK) {
        s = srt_plan_sync(p, err);
        if (s == SRT_OK && ct) {
            ct->release();
            ct->n = p->n;
            ct->bytes = SRT_RI_PATH16;
            ct->full = static_cast<srt_path *>(std::malloc(std::max<uint64_t>((uint64_t)p->n * p->n, 1) *
                                                           sizeof(srt_path)));
            if (!ct->full) {
                srt_plan_destroy(p);
                set_err(err, SRT_ERR_OOM, "out of host memory (routing table)");
                return SRT_ERR_OOM;
            }
            out = ct->full;
        }
        if (s == SRT_OK) s = srt_plan_fetch(p, out, min_latency_ns, err);
        if (s == SRT_OK && ct) {
            ct->diag.resize(p->n);
            for (uint32_t i = 0; i < p->n; ++i) ct->diag[i] = out[(uint64_t)i * p->n + i];
        }
    }
    tr.mark("e2e: build + fetch");
    // the device's loss range check (the host scan skipped it): a parse-time
    // error, so it wins over any error of the build itself
    join_loss_check(p);
    if (p->h_lossbad && s != SRT_ERR_HIP) {
        (void)hipStreamSynchronize(p->comm_stream);
        if (*p->h_lossbad != ~0ull) {
            s = SRT_ERR_INVALID;
            set_err(err, SRT_ERR_INVALID, "Edge 'packet_loss' is not in the range [0,1]");
        }
    }
    reap_async(p);  // teardown behind the return
    tr.mark("e2e: destroy queued");
    return s;
}

// srt_init: the HIP runtime on the device, the library's code objects (one
// kernel of each translation unit, which loads that unit's whole code object)
// and the pinned transfer staging
struct InitState {
    std::mutex m;
    std::thread th;
    bool pending = false;
    std::vector<int> done_dev;  // devices initialised
    srt_status last = SRT_OK;
    std::string msg;
};
InitState g_init;

// Exit while the async init runs.  glibc's exit() (also a return from main)
// first runs the EXITING thread's thread_local destructors, and only then the
// atexit / static-destructor list in reverse order of registration.  That
// list is no safe place to join: the init thread registers destructors of its
// own (the runtime's lazily built statics, code-object loaders) after any
// handler srt_init_async could register, so those would run first, under the
// still-running thread.  So srt_init_async plants a thread_local guard on the
// calling thread (Shadow's main) whose destructor joins the init: it runs
// before anything is destroyed.  On a thread that merely ends it also joins
// (that thread waits for the init; harmless).  The atexit join stays for a
// process that exits from another thread.
struct InitExitGuard {
    ~InitExitGuard() { srt::init_wait(); }
};
void join_init_at_exit() { srt::init_wait(); }

srt_status init_device(int device, std::string *msg) {
    int dev = device;
    if (dev < 0 && hipGetDevice(&dev) != hipSuccess) dev = 0;
    hipError_t e = hipSetDevice(dev);
    if (e == hipSuccess) e = hipFree(nullptr);  // creates the context
    if (e == hipSuccess) e = srt::preload_kernels();
    // the hardware queues behind a plan's streams (one normal, two high
    // priority): the runtime creates them on first use (~0.1 s) and keeps
    // them for later streams of the same priority
    if (e == hipSuccess) {
        int lo = 0, hi = 0;
        (void)hipDeviceGetStreamPriorityRange(&lo, &hi);
        hipStream_t s[3] = {nullptr, nullptr, nullptr};
        void *scratch = nullptr;
        e = hipMalloc(&scratch, 4096);
        if (e == hipSuccess) e = hipStreamCreateWithFlags(&s[0], hipStreamNonBlocking);
        if (e == hipSuccess) e = hipStreamCreateWithPriority(&s[1], hipStreamNonBlocking, hi);
        if (e == hipSuccess) e = hipStreamCreateWithPriority(&s[2], hipStreamNonBlocking, hi);
        for (int i = 0; i < 3 && e == hipSuccess; ++i) e = hipMemsetAsync(scratch, 0, 4096, s[i]);
        for (int i = 0; i < 3 && e == hipSuccess; ++i) e = hipStreamSynchronize(s[i]);
        for (int i = 0; i < 3; ++i)
            if (s[i]) (void)hipStreamDestroy(s[i]);
        if (scratch) (void)hipFree(scratch);
    }
    if (e == hipSuccess) {
        std::lock_guard<std::mutex> lk(g_pinned.m);
        if (!g_pinned.ensure(PINNED_BYTES)) e = hipErrorOutOfMemory;
    }
    if (e != hipSuccess) {
        *msg = std::string("srt_init: ") + hipGetErrorString(e);
        return SRT_ERR_HIP;
    }
    return SRT_OK;
}
}  // namespace

}  // extern "C"

namespace srt {
void cspan_begin(srt_plan *p) {
    if (!p->in_create) return;
    hipEvent_t e = nullptr;
    if (hipEventCreate(&e) != hipSuccess) return;
    (void)hipEventRecord(e, p->stream);
    p->cspan.push_back(e);
}
void cspan_end(srt_plan *p) {
    if (!p->in_create || p->cspan.size() % 2 == 0) return;
    hipEvent_t e = nullptr;
    if (hipEventCreate(&e) != hipSuccess) {
        (void)hipEventDestroy(p->cspan.back());
        p->cspan.pop_back();
        return;
    }
    (void)hipEventRecord(e, p->stream);
    p->cspan.push_back(e);
}
void init_wait() {
    std::thread t;
    {
        std::lock_guard<std::mutex> lk(g_init.m);
        if (!g_init.pending) return;
        t = std::move(g_init.th);
        g_init.pending = false;
    }
    if (t.joinable()) t.join();
}

srt_status routing_build(const srt_csr *g, const uint32_t *nodes, uint32_t n, const srt_opts *opts, CompactTable *t,
                         uint64_t *min_latency, srt_err *err) {
    return build_e2e(g, nodes, n, nullptr, t, min_latency, opts, err);
}
}  // namespace srt

extern "C" {

srt_status srt_compute_shortest_paths(const srt_csr *g, const uint32_t *nodes, uint32_t n,
                                      srt_path *out, uint64_t *min_latency_ns,
                                      const srt_opts *opts, srt_err *err) {
    return build_e2e(g, nodes, n, out, nullptr, min_latency_ns, opts, err);
}

srt_status srt_init(int device, srt_err *err) {
    clear_err(err);
    srt::init_wait();
    std::lock_guard<std::mutex> lk(g_init.m);
    int dev = device;
    if (dev < 0 && hipGetDevice(&dev) != hipSuccess) dev = 0;
    if (g_init.last != SRT_OK) {  // a failed async init
        const srt_status s = g_init.last;
        set_err(err, s, g_init.msg.c_str());
        g_init.last = SRT_OK;
        return s;
    }
    if (std::find(g_init.done_dev.begin(), g_init.done_dev.end(), dev) != g_init.done_dev.end()) return SRT_OK;
    std::string msg;
    const srt_status s = init_device(dev, &msg);
    if (s != SRT_OK) {
        set_err(err, s, msg.c_str());
        return s;
    }
    g_init.done_dev.push_back(dev);
    return SRT_OK;
}

void srt_init_wait(void) { srt::init_wait(); }

void srt_init_async(int device) {
    static std::once_flag reg;
    std::call_once(reg, [] {
        int count = 0;
        (void)hipGetDeviceCount(&count);
        std::atexit(join_init_at_exit);
    });
    static thread_local InitExitGuard guard;  // joins at this thread's exit / exit()
    (void)&guard;
    std::lock_guard<std::mutex> lk(g_init.m);
    if (g_init.pending) return;
    g_init.pending = true;
    g_init.th = std::thread([device] {
        std::string msg;
        int dev = device;
        if (dev < 0 && hipGetDevice(&dev) != hipSuccess) dev = 0;
        const srt_status s = init_device(dev, &msg);
        std::lock_guard<std::mutex> lk2(g_init.m);
        if (s == SRT_OK) g_init.done_dev.push_back(dev);
        else {
            g_init.last = s;
            g_init.msg = msg;
        }
    });
}

}  // extern "C"
