// hb_kernels.hpp -- CDNA4 (gfx950) kernels of the Swizzle hot path (templates;
// instantiated per limb count by hb_kern_nl*.hip, misc kernels in hb_kern_misc.hip).
//
//   hb_encode_kernel   tags of a run of blocks     (PySwizzle.py:296-309)
//   hb_prf_kernel      batched KeyedPRF.eval        (util.py:83-96)
//   hb_mont_kernel     x -> x R mod p (Montgomery form of alpha_j, v_i)
//   hb_wsum_kernel     per-thread partial sums of w_i * value(i) for prove /
//                      verify (PySwizzle.py:351-368, :388-394)
//   hb_sum_kernel      mod-p tree reduction of the partials
//   hb_fill_kernel     synthetic file bytes (SplitMix64), benches and tests
//
// PRF engine.  KeyedPRF.eval is rejection sampling (E[tries] = 2^bitlen(R)/R,
// up to 2): a lane-per-block loop where each lane retries until accepted would
// run every wave for the MAX of 64 geometric trip counts (~3x the mean).
// Instead each lane owns a job (block / PRF input) and the wave re-deals jobs
// after every try: lanes whose try was accepted finish their job and take the
// next ones from a wave-local pool refilled from a global counter
// (HB_QUEUE_CHUNK jobs per atomic).  Every try of every lane is useful work
// until the queue drains.  One try = nb CFB-8 steps = nb AES encryptions of
// which only byte 0 is used (hb_lane.hpp).
//
// The AES T tables live in LDS as a 64 KiB bank-replicated T0/T1 image
// (hb_lane.hpp, LaneTab): ds_read_b32 lookups are conflict-free for any
// indices, and the per-CU LDS rate (one wave-wide ds_read_b32 per 2 cycles)
// is the kernel's binding resource (roofline).
#pragma once
#include <hip/hip_runtime.h>
#include "hb_args.hpp"

#define HB_LDS_WORDS (HB_TAB_BYTES / 4)

// Expand the 256-entry global T0 into the replicated LDS image (hb_lane.hpp).
__device__ __forceinline__ void hb_fill_lds(u32 *lds, const u32 *t0) {
    // 16-byte writes: group g covers bytes 16g..16g+15 = one (table, entry)
    for (u32 g = threadIdx.x; g < HB_LDS_WORDS / 4; g += blockDim.x) {
        const u32 off = g * 16u;
        const u32 e = (off >> 8) & 0xffu, t = ((off >> 16) << 1) | ((off >> 7) & 1u);
        u32 v = t0[e];
        if (t) v = (v << (8 * t)) | (v >> (32 - 8 * t));
        reinterpret_cast<uint4 *>(lds)[g] = make_uint4(v, v, v, v);
    }
    __syncthreads();
}

__device__ __forceinline__ LaneTab hb_lane_tab(const u32 *lds) {
    const u32 r4 = (threadIdx.x & 31u) * 4u;
    return LaneTab{(const char *)lds, {r4, 128u + r4, 0x10000u | r4, 0x10000u | (128u + r4)}};
}

__device__ __forceinline__ u32 hb_lane_id() { return threadIdx.x & 63u; }

__device__ __forceinline__ u32 hb_mbcnt(u64 mask) {
    return __builtin_amdgcn_mbcnt_hi((u32)(mask >> 32), __builtin_amdgcn_mbcnt_lo((u32)mask, 0u));
}

__device__ __forceinline__ u64 hb_bcast64(u64 v) {
    u32 lo = __builtin_amdgcn_readfirstlane((u32)v);
    u32 hi = __builtin_amdgcn_readfirstlane((u32)(v >> 32));
    return ((u64)hi << 32) | lo;
}

// Wave-local job pool over a global counter.  All members are wave-uniform.
struct HbPool {
    u64 next, end, njobs;
    unsigned long long *counter;
    bool exhausted;

    // Lanes in `mask` (wave-uniform ballot) each want one job; returns whether
    // this lane (if `want`) got one, in `job`.
    __device__ __forceinline__ bool take(u64 mask, bool want, u64 &job) {
        const u32 need = (u32)__popcll(mask);
        const u32 rank = hb_mbcnt(mask);
        const u64 avail = end - next;
        u64 base2 = 0, got2 = 0;
        if (avail < need && !exhausted) {
            u64 b = 0;
            if (hb_lane_id() == 0) b = atomicAdd(counter, (unsigned long long)HB_QUEUE_CHUNK);
            b = hb_bcast64(b);
            if (b >= njobs) {
                exhausted = true;
            } else {
                base2 = b;
                got2 = njobs - b < (u64)HB_QUEUE_CHUNK ? njobs - b : (u64)HB_QUEUE_CHUNK;
            }
        }
        bool ok = false;
        if (want) {
            if ((u64)rank < avail) {
                job = next + rank;
                ok = true;
            } else if ((u64)rank - avail < got2) {
                job = base2 + ((u64)rank - avail);
                ok = true;
            }
        }
        if ((u64)need <= avail) {
            next += need;
        } else {
            const u64 used2 = (u64)need - avail < got2 ? (u64)need - avail : got2;
            next = base2 + used2;
            end = base2 + got2;
        }
        return ok;
    }
};

// The PRF engine: runs KeyedPRF.eval for every job of the queue and calls
// h.accept(job, value) once per job with the accepted value.  h.init(job, sr)
// sets the CFB-8 shift register a job starts from (zero for a fresh eval).
// MODE 0: KeyedPRF (util.py:83-96); MODE 1: the cxx prf (prf.hxx:125-176,
// hb_cxx_try), whose x is an unsigned int and which accepts after 81 tries.
template <int MODE>
__device__ __forceinline__ void hb_prf_digest(u64 x, u32 dig[8]) {
    if (MODE != 0) hb_sha256_le32((u32)x, dig);
    else hb_sha256_decimal(x, dig);
}

// The digest a job's PRF input hashes to: handlers with precomputed digests
// (hb_prf_eval_digests) provide digest(); the others hash x_of(job).
template <int MODE, class H>
__device__ __forceinline__ auto hb_job_digest(const H &h, u64 job, u32 dig[8], int)
    -> decltype(h.digest(job, dig), void()) {
    if (!h.digest(job, dig)) hb_prf_digest<MODE>(h.x_of(job), dig);
}
template <int MODE, class H>
__device__ __forceinline__ void hb_job_digest(const H &h, u64 job, u32 dig[8], long) {
    hb_prf_digest<MODE>(h.x_of(job), dig);
}

template <int NL, int NR, class H, int MODE = 0>
__device__ __forceinline__ void hb_engine(H &h, const LaneTab &L, const PrfParams<NL> &P,
                                          u64 njobs, unsigned long long *queue) {
    HbPool pool{0, 0, njobs, queue, false};
    u64 job = 0;
    bool active = pool.take(__ballot(1), true, job);
    u32 dig[8], sr[4] = {0, 0, 0, 0}, out[NL];
    if (active) {
        h.init(job, sr);
        hb_job_digest<MODE>(h, job, dig, 0);
    }
    u32 tries = 0, job_tries = 0, failed = 0;
    while (__ballot(active)) {
        u32 ok;
        if constexpr (MODE == 1) ok = hb_cxx_try<NL, NR>(L, P, sr, dig, out);
        else if constexpr (MODE == 2) ok = hb_cxx_try_bytes<NL, NR>(L, P, sr, dig, out, job_tries);
        else ok = hb_prf_try<NL, NR>(L, P, sr, dig, out);
        tries += active ? 1u : 0u;
        job_tries += 1u;
        if (MODE != 0 && job_tries >= HB_CXX_MAX_TRIES) ok = 1;   // `count++ < 80` (prf.hxx:142)
        const bool acc = active && ok;
        if (acc) h.accept(job, out);
        // Exit guarantee: a job still rejected after HB_MAX_TRIES tries
        // (probability <= 2^-HB_MAX_TRIES for any valid range) is dropped and
        // counted in queue[2]; the host reports it as an error.
        const bool give_up = active && !ok && job_tries >= HB_MAX_TRIES;
        failed += give_up ? 1u : 0u;
        const bool next = acc || give_up;
        const u64 m = __ballot(next);
        if (m) {
            u64 nj = 0;
            const bool got = pool.take(m, next, nj);
            if (next) {
                active = got;
                job = nj;
                job_tries = 0;
                if (got) {
                    h.init(job, sr);   // fresh cipher per eval (util.py:88) or a resumed stream
                    hb_job_digest<MODE>(h, job, dig, 0);
                }
            }
        }
    }
    // statistics: one atomic per wave
    for (int off = 32; off > 0; off >>= 1) {
        tries += __shfl_xor(tries, off);
        failed += __shfl_xor(failed, off);
    }
    if (hb_lane_id() == 0 && tries) atomicAdd(queue + 1, (unsigned long long)tries);
    if (hb_lane_id() == 0 && failed) atomicAdd(queue + 2, (unsigned long long)failed);
}

// ------------------------------------------------------------------ encode
// Minimum waves per SIMD requested from the register allocator: 4 (= one
// 1024-thread workgroup, 16 waves per CU, sharing one 128 KiB LDS table
// image) for primes up to 256 bits; wider primes keep the compiler's choice
// (they are not the benchmarked configuration).
template <int NL>
#ifndef HB_OCC8
#define HB_OCC8 4
#endif
struct HbEncodeOcc { static constexpr int v = NL <= 8 ? HB_OCC8 : 1; };


__device__ __forceinline__ void hb_zero_sr(u32 sr[4]) { sr[0] = sr[1] = sr[2] = sr[3] = 0; }

template <int NL, int ALIGN, int MODE = 0>
struct EncodeHandler {
    const EncodeArgs<NL> &A;
    __device__ __forceinline__ u64 x_of(u64 job) const { return A.block_base + job; }
    __device__ __forceinline__ void init(u64, u32 sr[4]) const { hb_zero_sr(sr); }
    __device__ __forceinline__ void accept(u64 job, const u32 F[NL]) const {
#if defined(HB_EXP_NO_MAC)
        hb_store_be<NL>(A.tags + job * (u64)A.tw, A.tw, F);
#else
        if (MODE == 1 && job * A.C >= A.len) {
            // cxx: no sector read -> sigma = f(chunk_id) without `%= p`
            // (shacham_waters_private.cxx:681-690; differs only if F >= p)
            hb_store_be<NL>(A.tags + job * (u64)A.tw, A.tw, F);
            return;
        }
        u32 tag[NL];
        hb_block_tag<NL, ALIGN>(A.data, A.len, job, A.C, A.ss, A.S, A.alpha_mont, A.mod, F, tag);
        hb_store_be<NL>(A.tags + job * (u64)A.tw, A.tw, tag);
#endif
    }
};

template <int NL, int NR, int ALIGN>
__global__ __launch_bounds__(HB_ENGINE_WG, HbEncodeOcc<NL>::v) void hb_encode_kernel(EncodeArgs<NL> A) {
    __shared__ __attribute__((aligned(16))) u32 lds[HB_LDS_WORDS];
    hb_fill_lds(lds, A.t0);
    const LaneTab L = hb_lane_tab(lds);
    EncodeHandler<NL, ALIGN> h{A};
    hb_engine<NL, NR>(h, L, A.prf, A.nblocks, A.queue);
}

// The cxx Swizzle encode (shacham_waters_private.cxx:638-702): the same
// engine and MAC with the cxx prf (CFB-128: nb/16 full AES per try instead of
// nb byte-0 AES).
template <int NL, int NR, int ALIGN>
__global__ __launch_bounds__(HB_ENGINE_WG, HbEncodeOcc<NL>::v) void hb_cxx_encode_kernel(EncodeArgs<NL> A) {
    __shared__ __attribute__((aligned(16))) u32 lds[HB_LDS_WORDS];
    hb_fill_lds(lds, A.t0);
    const LaneTab L = hb_lane_tab(lds);
    EncodeHandler<NL, ALIGN, 1> h{A};
    hb_engine<NL, NR, EncodeHandler<NL, ALIGN, 1>, 1>(h, L, A.prf, A.nblocks, A.queue);
}

// ------------------------------------------------------------------ two-pass encode
// The prefix image (hb_lane.hpp) turns the first 4 of the nb AES of a fresh
// eval into three byte loads, but only for a FIRST try: a lane re-dealt in the
// single-pass engine would still run in lockstep with lanes on later tries.
// So the encode splits by try:
//   pass 1 (hb_encode_first_kernel): every lane runs the first try of a fresh
//          block (nb - 4 AES); accepted blocks are tagged at once, rejected
//          ones (1 - p/2^bitlen(p) of them, 14 % for the bench prime) are
//          appended to the retry list with their shift register;
//   pass 2 (hb_encode_retry_kernel): the single-pass engine over the retry
//          list, resuming each stream where pass 1 left it.
// AES per block: nb (E[tries] - 1) + nb - 4 instead of nb E[tries].
template <int NR>
__global__ __launch_bounds__(HB_ENGINE_WG) void hb_prefix_kernel(PrefixArgs A) {
    __shared__ __attribute__((aligned(16))) u32 lds[HB_LDS_WORDS];
    hb_fill_lds(lds, A.t0);
    const LaneTab L = hb_lane_tab(lds);
    const u32 stride = gridDim.x * blockDim.x;
    for (u32 i = blockIdx.x * blockDim.x + threadIdx.x; i < HB_PFX_BYTES; i += stride)
        A.out[i] = (unsigned char)hb_aes_byte0<NR>(L, A.rk, 0u, 0u, 0u, hb_pfx_s3(i));
}

// End of one first try for one job slot of every lane (wave-uniform call):
// accepted blocks are tagged, rejected ones go to the retry list with their
// shift register.
template <int NL, int NR, int ALIGN, class H>
__device__ __forceinline__ void hb_first_finish(const EncodeArgs<NL> &A, const LaneTab &L, H &h, u64 job,
                                                bool active, u32 ok, u32 sr[4], u32 out[NL], u32 &tries,
                                                u32 &failed) {
    tries += active ? 1u : 0u;
    const u64 rej = __ballot(active && !ok);
    if (rej) {
        u64 base = 0;
        if (hb_lane_id() == 0) base = atomicAdd(A.retry_count, (unsigned long long)__popcll(rej));
        base = hb_bcast64(base);
        if (active && !ok) {
            const u64 slot = base + hb_mbcnt(rej);
            if (slot < A.retry_cap) {
                HbRetry *e = A.retry + slot;
                e->blk = job;
                *reinterpret_cast<uint4 *>(e->sr) = make_uint4(sr[0], sr[1], sr[2], sr[3]);
            } else {
                // retry list full (never at its sizing, see hb_runtime.cpp):
                // finish this eval in place
                u32 dig[8];
                hb_sha256_decimal(A.block_base + job, dig);
                u32 n = 1;
                while (!ok && n < HB_MAX_TRIES) {
                    ok = hb_prf_try<NL, NR>(L, A.prf, sr, dig, out);
                    ++n;
                    ++tries;
                }
                failed += ok ? 0u : 1u;
            }
        }
    }
    if (active && ok) h.accept(job, out);
}

// Blocks per lane per first-pass iteration.  Two independent evals whose AES
// interleave double the ds_read_b32 in flight per round (+11 % LDS lookup rate
// in isolation, scripts/ubench_aes.hip), but at 128 VGPRs the 256-bit encode
// spills and measured 933 vs 967 GiB/s at configs[2]: one by default.
#ifndef HB_FIRST_NJ
#define HB_FIRST_NJ 1
#endif
template <int NL>
struct HbFirstNJ { static constexpr int v = NL <= 8 ? HB_FIRST_NJ : 1; };

template <int NL, int NR, int ALIGN>
__global__ __launch_bounds__(HB_ENGINE_WG, HbEncodeOcc<NL>::v) void hb_encode_first_kernel(EncodeArgs<NL> A) {
    constexpr int NJ = HbFirstNJ<NL>::v;
    __shared__ __attribute__((aligned(16))) u32 lds[HB_LDS_WORDS];
    hb_fill_lds(lds, A.t0);
    const LaneTab L = hb_lane_tab(lds);
    EncodeHandler<NL, ALIGN> h{A};
    HbPool pool{0, 0, A.nblocks, A.queue, false};
    u32 tries = 0, failed = 0;
    for (;;) {
        u64 job0 = 0, job1 = 0;
        const bool act0 = pool.take(__ballot(1), true, job0);
        const bool act1 = NJ == 2 ? pool.take(__ballot(1), true, job1) : false;
        if (!__ballot(act0 || act1)) break;
        u32 out[NJ][NL], sr[NJ][4];
        u32 okm;
        {
            u32 dig[NJ][8];
            hb_sha256_decimal(A.block_base + job0, dig[0]);
            hb_prf_prefix<NL>(A.pfx, A.o0, A.prf, dig[0][0], sr[0], out[0]);
            if (NJ == 2) {
                hb_sha256_decimal(A.block_base + job1, dig[NJ - 1]);
                hb_prf_prefix<NL>(A.pfx, A.o0, A.prf, dig[NJ - 1][0], sr[NJ - 1], out[NJ - 1]);
            }
            okm = hb_prf_try_n<NL, NR, 1, NJ>(L, A.prf, sr, dig, out);
        }
        hb_first_finish<NL, NR, ALIGN>(A, L, h, job0, act0, okm & 1u, sr[0], out[0], tries, failed);
        if (NJ == 2)
            hb_first_finish<NL, NR, ALIGN>(A, L, h, job1, act1, (okm >> 1) & 1u, sr[NJ - 1], out[NJ - 1],
                                           tries, failed);
    }
    for (int off = 32; off > 0; off >>= 1) {
        tries += __shfl_xor(tries, off);
        failed += __shfl_xor(failed, off);
    }
    if (hb_lane_id() == 0 && tries) atomicAdd(A.queue + 1, (unsigned long long)tries);
    if (hb_lane_id() == 0 && failed) atomicAdd(A.queue + 2, (unsigned long long)failed);
}

template <int NL, int ALIGN>
struct RetryHandler {
    const EncodeArgs<NL> &A;
    __device__ __forceinline__ u64 x_of(u64 job) const { return A.block_base + A.retry[job].blk; }
    __device__ __forceinline__ void init(u64 job, u32 sr[4]) const {
        const uint4 v = *reinterpret_cast<const uint4 *>(A.retry[job].sr);
        sr[0] = v.x; sr[1] = v.y; sr[2] = v.z; sr[3] = v.w;
    }
    __device__ __forceinline__ void accept(u64 job, const u32 F[NL]) const {
        const u64 blk = A.retry[job].blk;
        u32 tag[NL];
        hb_block_tag<NL, ALIGN>(A.data, A.len, blk, A.C, A.ss, A.S, A.alpha_mont, A.mod, F, tag);
        hb_store_be<NL>(A.tags + blk * (u64)A.tw, A.tw, tag);
    }
};

template <int NL, int NR, int ALIGN>
__global__ __launch_bounds__(HB_ENGINE_WG, HbEncodeOcc<NL>::v) void hb_encode_retry_kernel(EncodeArgs<NL> A) {
    __shared__ __attribute__((aligned(16))) u32 lds[HB_LDS_WORDS];
    // pass 1 has completed (stream order): the count is final
    const u64 cnt = *(volatile unsigned long long *)A.retry_count;
    const u64 n = cnt < A.retry_cap ? cnt : A.retry_cap;
    if (n == 0) return;
    hb_fill_lds(lds, A.t0);
    const LaneTab L = hb_lane_tab(lds);
    RetryHandler<NL, ALIGN> h{A};
    hb_engine<NL, NR>(h, L, A.prf, n, A.queue);
}

// ------------------------------------------------------------------ PRF batch
template <int NL>
struct PrfHandler {
    const PrfArgs<NL> &A;
    __device__ __forceinline__ u64 x_of(u64 job) const { return A.xs ? A.xs[job] : A.x0 + job; }
    // SHA-256 digests supplied by the host (inputs outside [0, 2^64): the
    // reference hashes str(x) of any int, util.py:91)
    __device__ __forceinline__ bool digest(u64 job, u32 dig[8]) const {
        if (!A.digs) return false;
        for (int t = 0; t < 8; ++t) dig[t] = A.digs[job * 8 + t];
        return true;
    }
    __device__ __forceinline__ void init(u64, u32 sr[4]) const { hb_zero_sr(sr); }
    __device__ __forceinline__ void accept(u64 job, const u32 v[NL]) const {
        u32 *o = A.out + job * NL;
        for (int t = 0; t < NL; ++t) o[t] = v[t];
    }
};

template <int NL, int NR, int MODE>
__global__ __launch_bounds__(HB_ENGINE_WG) void hb_prf_kernel(PrfArgs<NL> A) {
    __shared__ __attribute__((aligned(16))) u32 lds[HB_LDS_WORDS];
    hb_fill_lds(lds, A.t0);
    const LaneTab L = hb_lane_tab(lds);
    PrfHandler<NL> h{A};
    hb_engine<NL, NR, PrfHandler<NL>, MODE>(h, L, A.prf, A.n, A.queue);
}

// ------------------------------------------------------------------ Montgomery
template <int NL>
__global__ __launch_bounds__(256) void hb_mont_kernel(MontArgs<NL> A) {
    const u64 i = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= A.n) return;
    u32 x[NL], y[NL];
    for (int t = 0; t < NL; ++t) x[t] = A.in[i * NL + t];
    hb_to_mont<NL>(x, A.r2, A.mod, y);
    for (int t = 0; t < NL; ++t) A.out[i * NL + t] = y[t];
}

// ------------------------------------------------------------------ prove / verify sums
template <int NL, int ALIGN>
__device__ __forceinline__ void hb_sector_value(const unsigned char *data, u64 len, u64 pos,
                                                u32 ss, u32 m[NL]) {
    if (pos >= len) {
        for (int t = 0; t < NL; ++t) m[t] = 0;
    } else if (pos + ss <= len) {
        if (ALIGN == 16) hb_load_full16<NL>(data, pos, m);
        else hb_load_be_bytes<NL>(data, pos, ss, m);
    } else {
        hb_load_be_bytes<NL>(data, pos, (u32)(len - pos), m);
    }
}

template <int NL, int ALIGN>
__global__ __launch_bounds__(256) void hb_wsum_kernel(WsumArgs<NL> A) {
    const u32 col = blockIdx.y;
    const u64 tid = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    const u64 nthreads = (u64)gridDim.x * blockDim.x;
    u32 acc[2 * NL + 1];
    for (int t = 0; t <= 2 * NL; ++t) acc[t] = 0;
    u32 m[NL];
    for (u64 i = tid; i < A.nterms; i += nthreads) {
        if (A.mode == 1) {
            for (int t = 0; t < NL; ++t) m[t] = A.vals[i * NL + t];
        } else {
            const bool gathered = A.mode == 2;
            const u64 blk = gathered ? i : A.idx[i];
            if (col < A.S) {
                const u64 blen = gathered ? A.blen[i] : A.len;
                const u64 base = gathered ? i * A.C : A.wrap32 ? (u64)(u32)(blk * A.C) : blk * A.C;
                const u64 pos = base + (u64)col * A.ss;
                const u64 end = gathered ? base + blen : A.len;
                hb_sector_value<NL, ALIGN>(A.data, end, pos, A.ss, m);
            } else {
                hb_load_be_bytes<NL>(A.tags, blk * A.tw, A.tw, m);
            }
        }
        hb_mac<NL>(acc, A.w + i * NL, m);
    }
    u32 v[NL + 1], r[NL];
    hb_redc<NL>(acc, A.mod, v);
    hb_reduce_small<NL>(v, A.mod, r);
    u32 *o = A.partials + ((u64)col * nthreads + tid) * NL;
    for (int t = 0; t < NL; ++t) o[t] = r[t];
}

// one workgroup per column: sum nparts residues mod p
template <int NL>
__global__ __launch_bounds__(256) void hb_sum_kernel(SumArgs<NL> A) {
    __shared__ u32 sh[256 * NL];
    const u32 col = blockIdx.x;
    u32 v[NL + 1];
    for (int t = 0; t <= NL; ++t) v[t] = 0;
    for (u32 k = threadIdx.x; k < A.nparts; k += blockDim.x) {
        const u32 *x = A.partials + ((u64)col * A.nparts + k) * NL;
        u64 c = 0;
        for (int t = 0; t < NL; ++t) {
            c += (u64)v[t] + x[t];
            v[t] = (u32)c;
            c >>= 32;
        }
        v[NL] += (u32)c;
    }
    u32 r[NL];
    hb_reduce_small<NL>(v, A.mod, r);
    for (int t = 0; t < NL; ++t) sh[threadIdx.x * NL + t] = r[t];
    __syncthreads();
    for (u32 s = blockDim.x / 2; s > 0; s >>= 1) {
        if (threadIdx.x < s) {
            u32 w[NL + 1];
            u64 c = 0;
            for (int t = 0; t < NL; ++t) {
                c += (u64)sh[threadIdx.x * NL + t] + sh[(threadIdx.x + s) * NL + t];
                w[t] = (u32)c;
                c >>= 32;
            }
            w[NL] = (u32)c;
            hb_reduce_small<NL>(w, A.mod, r);
            for (int t = 0; t < NL; ++t) sh[threadIdx.x * NL + t] = r[t];
        }
        __syncthreads();
    }
    if (threadIdx.x < NL) A.out[col * NL + threadIdx.x] = sh[threadIdx.x];
}

// ------------------------------------------------------------------ launchers
// Plain C++ entry points for hb_runtime.cpp (explicit instantiation per
// limb count NL, AES rounds NR and sector alignment class).
// pass: 0 = single-pass engine, 1 = first tries (prefix image), 2 = retry list,
// 3 = cxx prf encode
template <int NL>
hipError_t hb_launch_encode(const EncodeArgs<NL> &A, int nr, int align, int pass, int grid, hipStream_t s) {
    dim3 g(grid), b(HB_ENGINE_WG);
#define HB_ENC(K, NRV, AL) hipLaunchKernelGGL((K<NL, NRV, AL>), g, b, 0, s, A)
#define HB_ENC_NR(K, AL) \
    do { if (nr == 14) HB_ENC(K, 14, AL); else if (nr == 12) HB_ENC(K, 12, AL); else HB_ENC(K, 10, AL); } while (0)
#define HB_ENC_AL(K) do { if (align == 16) HB_ENC_NR(K, 16); else HB_ENC_NR(K, 1); } while (0)
    if (pass == 1) HB_ENC_AL(hb_encode_first_kernel);
    else if (pass == 2) HB_ENC_AL(hb_encode_retry_kernel);
    else if (pass == 3) HB_ENC_AL(hb_cxx_encode_kernel);
    else HB_ENC_AL(hb_encode_kernel);
#undef HB_ENC_AL
#undef HB_ENC_NR
#undef HB_ENC
    return hipGetLastError();
}


// mode 0: KeyedPRF, 1: cxx prf (ByteCount(limit) % 16 == 0), 2: cxx prf (any limit)
template <int NL>
hipError_t hb_launch_prf(const PrfArgs<NL> &A, int nr, int mode, int grid, hipStream_t s) {
    dim3 g(grid), b(HB_ENGINE_WG);
#define HB_PRF_NR(M)                                                               \
    do {                                                                           \
        if (nr == 14) hipLaunchKernelGGL((hb_prf_kernel<NL, 14, M>), g, b, 0, s, A); \
        else if (nr == 12) hipLaunchKernelGGL((hb_prf_kernel<NL, 12, M>), g, b, 0, s, A); \
        else hipLaunchKernelGGL((hb_prf_kernel<NL, 10, M>), g, b, 0, s, A);       \
    } while (0)
    if (mode == 1) {
        if constexpr (NL >= 4) HB_PRF_NR(1);   // cxx limits are >= 16 bytes
        else return hipErrorInvalidValue;
    } else if (mode == 2) {
        HB_PRF_NR(2);
    } else {
        HB_PRF_NR(0);
    }
#undef HB_PRF_NR
    return hipGetLastError();
}

template <int NL>
hipError_t hb_launch_mont(const MontArgs<NL> &A, hipStream_t s) {
    const u64 grid = (A.n + 255) / 256;
    hipLaunchKernelGGL((hb_mont_kernel<NL>), dim3((u32)grid), dim3(256), 0, s, A);
    return hipGetLastError();
}

template <int NL>
hipError_t hb_launch_wsum(const WsumArgs<NL> &A, int align, int gridx, hipStream_t s) {
    dim3 g(gridx, A.ncols), b(256);
    if (align == 16) hipLaunchKernelGGL((hb_wsum_kernel<NL, 16>), g, b, 0, s, A);
    else hipLaunchKernelGGL((hb_wsum_kernel<NL, 1>), g, b, 0, s, A);
    return hipGetLastError();
}

template <int NL>
hipError_t hb_launch_sum(const SumArgs<NL> &A, int ncols, hipStream_t s) {
    hipLaunchKernelGGL((hb_sum_kernel<NL>), dim3(ncols), dim3(256), 0, s, A);
    return hipGetLastError();
}

#define HB_INST(NL)                                                                              \
    template hipError_t hb_launch_encode<NL>(const EncodeArgs<NL> &, int, int, int, int, hipStream_t); \
    template hipError_t hb_launch_prf<NL>(const PrfArgs<NL> &, int, int, int, hipStream_t);      \
    template hipError_t hb_launch_mont<NL>(const MontArgs<NL> &, hipStream_t);                   \
    template hipError_t hb_launch_wsum<NL>(const WsumArgs<NL> &, int, int, hipStream_t);         \
    template hipError_t hb_launch_sum<NL>(const SumArgs<NL> &, int, hipStream_t);
