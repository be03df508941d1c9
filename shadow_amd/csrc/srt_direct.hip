// srt_direct.hip -- use_shortest_path = false: the table is the unique direct
// edge between every ordered pair of in-use nodes.
//
// Replaces NetworkGraph::get_direct_paths (src/main/network/graph/mod.rs:230-252)
// and its per-pair get_edge_weight/edges_connecting walk (mod.rs:256-293): one
// scatter pass over the adjacency of the in-use rows counts and records the
// edge of every pair, then the first pair (in the reference's iteration order:
// source-major over the caller's node list) whose count != 1 is reported with
// the reference's error text.
#include <cstdio>
#include <cstring>
#include <vector>

#include "srt_internal.h"

namespace {

__global__ void direct_scatter_kernel(const uint64_t *__restrict__ row_ptr,
                                      const uint32_t *__restrict__ col,
                                      const uint64_t *__restrict__ lat,
                                      const float *__restrict__ loss,
                                      const uint32_t *__restrict__ nodes,
                                      const int32_t *__restrict__ pos, uint32_t n,
                                      uint32_t *__restrict__ count, uint64_t *__restrict__ out_lat,
                                      float *__restrict__ out_loss) {
    const uint32_t wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t nwaves = (gridDim.x * blockDim.x) >> 6;
    for (uint32_t i = wave; i < n; i += nwaves) {
        const uint32_t u = nodes[i];
        for (uint64_t k = row_ptr[u] + lane; k < row_ptr[u + 1]; k += 64) {
            const int32_t j = pos[col[k]];
            if (j < 0) continue;
            const uint64_t o = (uint64_t)i * n + (uint32_t)j;
            atomicAdd(&count[o], 1u);
            out_lat[o] = lat[k];
            out_loss[o] = loss[k];
        }
    }
}

// first bad pair (min flat index) and min latency over good pairs
__global__ void direct_check_kernel(const uint32_t *__restrict__ count,
                                    const uint64_t *__restrict__ out_lat, uint64_t total,
                                    unsigned long long *stats) {
    unsigned long long first_bad = ~0ull, mn = ~0ull;
    for (uint64_t e = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; e < total;
         e += (uint64_t)gridDim.x * blockDim.x) {
        if (count[e] != 1) {
            if (e < first_bad) first_bad = e;
        } else if (out_lat[e] < mn) {
            mn = out_lat[e];
        }
    }
    for (int off = 32; off > 0; off >>= 1) {
        const unsigned long long a = __shfl_xor(first_bad, off), b = __shfl_xor(mn, off);
        first_bad = a < first_bad ? a : first_bad;
        mn = b < mn ? b : mn;
    }
    if ((threadIdx.x & 63) == 0) {
        atomicMin(&stats[0], mn);
        atomicMin(&stats[1], first_bad);
    }
}

__global__ void direct_init_stats(unsigned long long *stats) {
    stats[0] = ~0ull;
    stats[1] = ~0ull;
}

__global__ void direct_pack_kernel(const uint64_t *__restrict__ lat, const float *__restrict__ loss,
                                   srt_path *__restrict__ out, uint64_t total) {
    for (uint64_t e = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; e < total;
         e += (uint64_t)gridDim.x * blockDim.x) {
        srt_path p;
        p.latency_ns = lat[e];
        p.packet_loss = loss[e];
        p._pad = 0;
        out[e] = p;
    }
}

struct DevBuf {
    void *p = nullptr;
    ~DevBuf() {
        if (p) (void)hipFree(p);
    }
    hipError_t alloc(size_t bytes) { return hipMalloc(&p, bytes ? bytes : 1); }
};

}  // namespace

namespace srt {
// srt_init: loads this unit's code object (srt::preload_kernels)
hipError_t preload_direct() {
    hipFuncAttributes a;
    return hipFuncGetAttributes(&a, reinterpret_cast<const void *>(&direct_init_stats));
}
}  // namespace srt

extern "C" srt_status srt_get_direct_paths(const srt_csr *g, const uint32_t *nodes, uint32_t n,
                                           srt_path *out, uint64_t *min_latency_ns,
                                           const srt_opts *opts, srt_err *err) {
    srt::init_wait();  // a pending srt_init_async finishes first
    if (err) std::memset(err, 0, sizeof *err);
    auto fail = [&](int code, const char *msg) {
        if (err) {
            err->code = code;
            std::snprintf(err->msg, sizeof err->msg, "%s", msg);
        }
        return (srt_status)code;
    };
    if (!g || (n && (!nodes || !out)) || !g->row_ptr) return fail(SRT_ERR_INVALID, "null argument");
    std::vector<int32_t> pos(g->n_nodes, -1);
    for (uint32_t i = 0; i < n; ++i) {
        if (nodes[i] >= g->n_nodes || pos[nodes[i]] >= 0)
            return fail(SRT_ERR_INVALID, "in-use node list has an out-of-range or duplicate NodeIndex");
        pos[nodes[i]] = (int32_t)i;
    }
    if (n == 0) {
        if (min_latency_ns) *min_latency_ns = ~0ull;
        return SRT_OK;
    }
    int dev = opts && opts->device >= 0 ? opts->device : -1;
    if (dev >= 0 && hipSetDevice(dev) != hipSuccess) return fail(SRT_ERR_HIP, "hipSetDevice failed");
    hipStream_t s;
    if (hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess)
        return fail(SRT_ERR_HIP, "hipStreamCreate failed");
    const uint64_t total = (uint64_t)n * n;
    DevBuf row_ptr, col, lat, loss, dnodes, dpos, count, olat, oloss, stats, pack;
    srt_status rc = SRT_OK;
    do {
        if (row_ptr.alloc(((size_t)g->n_nodes + 1) * 8) || col.alloc(g->n_adj * 4) ||
            lat.alloc(g->n_adj * 8) || loss.alloc(g->n_adj * 4) || dnodes.alloc((size_t)n * 4) ||
            dpos.alloc((size_t)g->n_nodes * 4) || count.alloc(total * 4) || olat.alloc(total * 8) ||
            oloss.alloc(total * 4) || stats.alloc(16) || pack.alloc(total * sizeof(srt_path))) {
            rc = fail(SRT_ERR_OOM, "hipMalloc failed");
            break;
        }
        hipMemcpyAsync(row_ptr.p, g->row_ptr, ((size_t)g->n_nodes + 1) * 8, hipMemcpyHostToDevice, s);
        if (g->n_adj) {
            hipMemcpyAsync(col.p, g->col, g->n_adj * 4, hipMemcpyHostToDevice, s);
            hipMemcpyAsync(lat.p, g->lat_ns, g->n_adj * 8, hipMemcpyHostToDevice, s);
            hipMemcpyAsync(loss.p, g->loss, g->n_adj * 4, hipMemcpyHostToDevice, s);
        }
        hipMemcpyAsync(dnodes.p, nodes, (size_t)n * 4, hipMemcpyHostToDevice, s);
        hipMemcpyAsync(dpos.p, pos.data(), (size_t)g->n_nodes * 4, hipMemcpyHostToDevice, s);
        hipMemsetAsync(count.p, 0, total * 4, s);
        hipLaunchKernelGGL(direct_scatter_kernel, dim3(1024), dim3(256), 0, s,
                           (const uint64_t *)row_ptr.p, (const uint32_t *)col.p, (const uint64_t *)lat.p,
                           (const float *)loss.p, (const uint32_t *)dnodes.p, (const int32_t *)dpos.p, n,
                           (uint32_t *)count.p, (uint64_t *)olat.p, (float *)oloss.p);
        hipLaunchKernelGGL(direct_init_stats, dim3(1), dim3(1), 0, s, (unsigned long long *)stats.p);
        hipLaunchKernelGGL(direct_check_kernel, dim3(1024), dim3(256), 0, s, (const uint32_t *)count.p,
                           (const uint64_t *)olat.p, total, (unsigned long long *)stats.p);
        unsigned long long hs[2];
        hipMemcpyAsync(hs, stats.p, 16, hipMemcpyDeviceToHost, s);
        if (hipStreamSynchronize(s) != hipSuccess) {
            rc = fail(SRT_ERR_HIP, "direct-path kernels failed");
            break;
        }
        if (hs[1] != ~0ull) {
            uint32_t c;
            hipMemcpy(&c, (uint32_t *)count.p + hs[1], 4, hipMemcpyDeviceToHost);
            const uint32_t a = nodes[hs[1] / n], b = nodes[hs[1] % n];
            const uint32_t aid = g->node_ids ? g->node_ids[a] : a, bid = g->node_ids ? g->node_ids[b] : b;
            char buf[160];
            std::snprintf(buf, sizeof buf,
                          c == 0 ? "No edge connecting node %u to %u" : "More than one edge connecting node %u to %u",
                          aid, bid);
            rc = fail(c == 0 ? SRT_ERR_NO_EDGE : SRT_ERR_MULTI_EDGE, buf);
            if (err) {
                err->a_id = aid;
                err->b_id = bid;
            }
            break;
        }
        if (min_latency_ns) *min_latency_ns = hs[0];
        hipLaunchKernelGGL(direct_pack_kernel, dim3(1024), dim3(256), 0, s, (const uint64_t *)olat.p,
                           (const float *)oloss.p, (srt_path *)pack.p, total);
        hipMemcpyAsync(out, pack.p, total * sizeof(srt_path), hipMemcpyDeviceToHost, s);
        if (hipStreamSynchronize(s) != hipSuccess) rc = fail(SRT_ERR_HIP, "download failed");
    } while (0);
    (void)hipStreamDestroy(s);
    return rc;
}
