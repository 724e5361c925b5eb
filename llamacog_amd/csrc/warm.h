// warm.h — Infinity-Cache warming of upcoming decode weights.
//
// A batch-1 decode step alternates weight-streaming mat-vecs with latency-bound kernels
// (RMS norm + quantize, flash attention, the FFN product + quantize) that keep a few CUs busy
// for 3-10 us while HBM sits idle.  Those kernels carry extra "warm" workgroups that read the
// next mat-vecs' weight bytes HBM -> LDS (and discard them): the lines land in the 256 MiB
// die-level Infinity Cache, so the mat-vec that follows streams them on-die instead of from
// HBM (measured: the 33 MB down projection 11.7 -> 8.4 us, the 9.4 MB output projection
// 6.1 -> 3.9 us, scripts/probe_mall.py).  A line stays resident while the bytes touched in
// between stay under ~256 MiB (MI355X_MICROARCH.md, Infinity Cache); the planner never runs
// further ahead than the next few mat-vecs.  Every weight byte is still read from HBM once
// per token; the warm only moves the read into the idle window, and never changes a result.
#pragma once

#include "common.h"

namespace mi355x {

constexpr int WARM_MAXSEG = 4;

// up to WARM_MAXSEG byte ranges (whole KiB) of device memory, streamed by nwg workgroups
// appended to a kernel's own grid
struct warm_spec {
    const uint8_t * p[WARM_MAXSEG];
    int64_t         n[WARM_MAXSEG];
    int             nseg;
    int             nwg;
};

enum warm_kind { WARM_NORM = 0, WARM_FA = 1, WARM_MULQ = 2, WARM_NKIND = 3 };

typedef __attribute__((address_space(3))) void * warm_lds_t;

// Workgroup `wg` of the warm grid streams its share of the ranges in 1 KiB wave-instructions
// (global_load_lds, 16 B per lane, no VGPRs, default cache policy so the lines allocate in the
// Infinity Cache): wave-chunks are dealt round-robin over every wave of the warm grid, and the
// vmcnt scoreboard keeps up to 63 KiB in flight per wave without a wait.  `lds` = 1 KiB of
// scratch LDS per wave (lds_waves of them; waves beyond share).
__device__ __forceinline__ void warm_run(const warm_spec & w, int wg, uint8_t * lds, int lds_waves) {
    const int nwaves = blockDim.x >> 6;
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int64_t gw = (int64_t) wg * nwaves + wave;
    const int64_t stride = (int64_t) w.nwg * nwaves;
    uint8_t * dst = lds + 1024 * (wave % lds_waves);
#pragma unroll 1
    for (int s = 0; s < WARM_MAXSEG; ++s) {
        if (s >= w.nseg) break;
        const uint8_t * base = w.p[s];
        const int64_t nchunk = w.n[s] >> 10;
#pragma unroll 4
        for (int64_t c = gw; c < nchunk; c += stride) {
            __builtin_amdgcn_global_load_lds((const void *) (base + (c << 10) + 16 * lane), (warm_lds_t) dst, 16, 0, 0);
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

}  // namespace mi355x
