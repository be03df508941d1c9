// srt_scan.h -- the host pass over the borrowed CSR (srt_scan.cpp): the
// edge-attribute checks, self-loops and key-proof statistics of plan
// creation.  Plain C++ (no HIP): tools/scan_bench.cpp times it on the CPU.
#pragma once

#include <cstdint>
#include <vector>

#include "../../include/srt.h"

namespace srt {

struct CsrStats {
    uint64_t gcd = 0, maxlat = 0, selfloops = 0;
    uint64_t zero_k = ~0ull, badloss_k = ~0ull, badcol_k = ~0ull;
    bool unique = true, complete = true;
    // every row is exactly the entries 0 .. V-1 in order (complete graphs as
    // Shadow writes them): entry (u, v) sits at u * V + v
    bool ident = true;
    // symmetry fingerprint for the family price: sums over entries (u, v, l)
    // of u*(v*v + l) and of v*(u*u + l) (mod 2^32) -- equal for every graph
    // whose entry multiset is closed under (u, v, l) -> (v, u, l)
    uint64_t sym_a = 0, sym_b = 0;
    std::vector<uint32_t> sl_cnt;    // per node: self-loop entries
    std::vector<uint64_t> sl_first;  // per node: first self-loop entry
};

// host threads for a pass over `work` entries (the job's CPU share:
// OMP_NUM_THREADS / SRT_HOST_THREADS, at most 32; 1 below 1 Mi)
int host_threads(uint64_t work);

// Rows [r0, r1) into the thread's accumulator st (sl_cnt / sl_first of the
// rows go to out).  Optional, for the piece-pipelined upload: lat32 (the
// rows' latencies as u32, indexed from entry k_base; *lat_over set when one
// does not fit) and *identity (cleared unless every row is exactly the
// entries 0 .. V-1 in order, so col need not be uploaded).  check_loss
// false: the losses are left to the device (end-to-end builds check them on
// the GPU as they are uploaded; badloss_k stays unset).
void scan_rows(const srt_csr *g, uint32_t r0, uint32_t r1, CsrStats &st, CsrStats *out, uint32_t *lat32 = nullptr,
               uint64_t k_base = 0, bool *lat_over = nullptr, bool *identity = nullptr, bool check_loss = true);

// per-thread accumulators into out
void merge_stats(const std::vector<CsrStats> &part, uint32_t V, CsrStats *out);

// the whole CSR on host_threads(n_adj) threads
void csr_scan(const srt_csr *g, CsrStats *out, bool check_loss = true);

// the first entry whose loss is outside [0, 1] (~0 if none), on host threads
uint64_t first_bad_loss(const srt_csr *g);

// loss bits valid: +0 .. 1.0f, or -0.0f (IEEE >= 0 holds for it)
inline bool loss_bits_bad(uint32_t q) { return q > 0x3f800000u && q != 0x80000000u; }

}  // namespace srt
