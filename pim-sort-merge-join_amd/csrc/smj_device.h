// smj_device.h -- device helpers shared by the HIP kernel files
// (smj_kernels.hip: LSD radix passes + merge-path join; smj_msd.hip: the MSD
// sample-sort pipeline).  gfx950 only: wave64 DPP scans, v_bitop3, mbcnt.
#pragma once

#include "smj_internal.h"

namespace smj {

typedef long long i64x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ uint64_t biased(int64_t k) { return (uint64_t)k ^ 0x8000000000000000ull; }

template <int COLS>
__device__ __forceinline__ void load_row(const int64_t *__restrict__ p, int64_t (&r)[COLS]) {
    if constexpr (COLS % 2 == 0) {
        const i64x2 *q = reinterpret_cast<const i64x2 *>(p);
#pragma unroll
        for (int c = 0; c < COLS / 2; c++) {
            i64x2 t = q[c];
            r[2 * c] = t.x;
            r[2 * c + 1] = t.y;
        }
    } else {
#pragma unroll
        for (int c = 0; c < COLS; c++) r[c] = p[c];
    }
}

// load_row with nontemporal (streaming) loads
template <int COLS>
__device__ __forceinline__ void load_row_nt(const int64_t *__restrict__ p, int64_t (&r)[COLS]) {
    if constexpr (COLS % 2 == 0) {
        const i64x2 *q = reinterpret_cast<const i64x2 *>(p);
#pragma unroll
        for (int c = 0; c < COLS / 2; c++) {
            const i64x2 t = __builtin_nontemporal_load(q + c);
            r[2 * c] = t.x;
            r[2 * c + 1] = t.y;
        }
    } else {
#pragma unroll
        for (int c = 0; c < COLS; c++) r[c] = __builtin_nontemporal_load(p + c);
    }
}

// store_row with nontemporal (streaming) stores: for tiles written once and
// read back only by a later pass, after gigabytes of other traffic
template <int COLS>
__device__ __forceinline__ void store_row_nt(int64_t *__restrict__ p, const int64_t (&r)[COLS]) {
    if constexpr (COLS % 2 == 0) {
        i64x2 *q = reinterpret_cast<i64x2 *>(p);
#pragma unroll
        for (int c = 0; c < COLS / 2; c++) {
            i64x2 t;
            t.x = r[2 * c];
            t.y = r[2 * c + 1];
            __builtin_nontemporal_store(t, q + c);
        }
    } else {
#pragma unroll
        for (int c = 0; c < COLS; c++) __builtin_nontemporal_store(r[c], p + c);
    }
}

template <int COLS>
__device__ __forceinline__ void store_row(int64_t *__restrict__ p, const int64_t (&r)[COLS]) {
    if constexpr (COLS % 2 == 0) {
        i64x2 *q = reinterpret_cast<i64x2 *>(p);
#pragma unroll
        for (int c = 0; c < COLS / 2; c++) {
            i64x2 t;
            t.x = r[2 * c];
            t.y = r[2 * c + 1];
            q[c] = t;
        }
    } else {
#pragma unroll
        for (int c = 0; c < COLS; c++) p[c] = r[c];
    }
}

// r[col] with a run-time col.  Written as an and/or of per-column masks:
// the equivalent select chain is pattern-matched by hipcc into an indexed
// access, which demotes the whole row array to scratch memory.
template <int COLS>
__device__ __forceinline__ int64_t pick(const int64_t (&r)[COLS], int col) {
    if constexpr (COLS == 1) {
        return r[0];
    } else if constexpr (COLS == 2) {
        return col ? r[1] : r[0];  // one uniform select: two v_cndmask
    } else {
        int64_t v = 0;
#pragma unroll
        for (int c = 0; c < COLS; c++) v |= r[c] & -(int64_t)(col == c);
        return v;
    }
}

__device__ __forceinline__ uint32_t ld_status(const uint32_t *p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_status(uint32_t *p, uint32_t v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Inclusive wave64 scan on DPP (row_shr 1/2/4/8 inside each row of 16
// lanes, then row_bcast:15 / row_bcast:31 across rows): VALU-only, no LDS
// permutes.  `lane` is unused; kept for call-site symmetry.
__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t v, int lane) {
    (void)lane;
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xf, 0xf, false);  // row_shr:1
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xf, 0xf, false);  // row_shr:2
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xf, 0xf, false);  // row_shr:4
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xf, 0xf, false);  // row_shr:8
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xa, 0xf, false);  // row_bcast:15
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xc, 0xf, false);  // row_bcast:31
    return v;
}

// inclusive max over lanes 0..lane (lane 63: the wave's max), the DPP
// pattern of wave_incl_scan (unsigned; 0 is the identity)
__device__ __forceinline__ uint32_t wave_incl_max(uint32_t v) {
    v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xf, 0xf, false));
    v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xf, 0xf, false));
    v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xf, 0xf, false));
    v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xf, 0xf, false));
    v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xa, 0xf, false));
    v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xc, 0xf, false));
    return v;
}

// a wave zeroes its own row of digit counters
template <int RADIX>
__device__ __forceinline__ void zero_counters(uint32_t *wc, int lane) {
    if constexpr (RADIX % 4 == 0) {
        for (int i = lane; i < RADIX / 4; i += 64) reinterpret_cast<uint4 *>(wc)[i] = make_uint4(0, 0, 0, 0);
    } else {
        for (int i = lane; i < RADIX; i += 64) wc[i] = 0;
    }
}

// p &= ~(ballot ^ s) on one 32-bit half (s = 0 or ~0: this lane's bit)
__device__ __forceinline__ uint32_t peer_fold(uint32_t p, uint32_t ballot_half, uint32_t s) {
    return __builtin_amdgcn_bitop3_b32(p, ballot_half, s, 0x90);
}


#define SMJ_COLS_SWITCH(cols, ...)                    \
    switch (cols) {                                   \
    case 1: { constexpr int C = 1; __VA_ARGS__; } break; \
    case 2: { constexpr int C = 2; __VA_ARGS__; } break; \
    case 3: { constexpr int C = 3; __VA_ARGS__; } break; \
    case 4: { constexpr int C = 4; __VA_ARGS__; } break; \
    case 5: { constexpr int C = 5; __VA_ARGS__; } break; \
    case 6: { constexpr int C = 6; __VA_ARGS__; } break; \
    case 7: { constexpr int C = 7; __VA_ARGS__; } break; \
    case 8: { constexpr int C = 8; __VA_ARGS__; } break; \
    default: return hipErrorInvalidValue;             \
    }

static inline unsigned blocks_for(int64_t n, int64_t per) { return (unsigned)((n + per - 1) / per); }

}  // namespace smj
