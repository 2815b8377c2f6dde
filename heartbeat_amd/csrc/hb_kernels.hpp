// hb_kernels.hpp -- CDNA4 (gfx950) kernels of the Swizzle hot path (templates;
// instantiated per limb count by hb_kern_nl*.hip, misc kernels in hb_kern_misc.hip).
//
//   hb_encode_kernel   tags of a run of blocks     (PySwizzle.py:296-309)
//   hb_prf_kernel      batched KeyedPRF.eval        (util.py:83-96)
//   hb_mont_kernel     x -> x R mod p (Montgomery form of alpha_j, v_i)
//   hb_prove_prf_kernel  prove stage 1: index and v PRFs of a challenge
//   hb_wsum_kernel     weighted sums sum_i w_i * value(i) mod p for prove /
//                      verify (PySwizzle.py:351-368, :388-394), finished in
//                      the same launch by the last workgroup of each column
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
// The AES T tables live in LDS as a 128 KiB bank-replicated image of the four
// tables T0..T3 (hb_lane.hpp, LaneTab): ds_read_b32 lookups are conflict-free
// for any indices.  The per-CU LDS rate (one wave-wide ds_read_b32 per 2
// cycles) and the VALU issue rate (address v_perm, v_bitop3 XORs, SHA-256, CFB
// register) bind the encode together (PMC counters).
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

__device__ __forceinline__ u64 hb_qchunk(u64 q) { return q ? q : (u64)HB_QUEUE_CHUNK; }

// Wave-local job pool over a global counter.  All members are wave-uniform.
struct HbPool {
    u64 next, end, njobs;
    unsigned long long *counter;
    bool exhausted;
    u64 chunk;   // jobs per refill (HB_QUEUE_CHUNK; 64 for small latency-bound launches)

    // Lanes in `mask` (wave-uniform ballot) each want one job; returns whether
    // this lane (if `want`) got one, in `job`.
    __device__ __forceinline__ bool take(u64 mask, bool want, u64 &job) {
        const u32 need = (u32)__popcll(mask);
        const u32 rank = hb_mbcnt(mask);
        const u64 avail = end - next;
        u64 base2 = 0, got2 = 0;
        if (avail < need && !exhausted) {
            u64 b = 0;
            if (hb_lane_id() == 0) b = atomicAdd(counter, (unsigned long long)chunk);
            b = hb_bcast64(b);
            if (b >= njobs) {
                exhausted = true;
            } else {
                base2 = b;
                got2 = njobs - b < chunk ? njobs - b : chunk;
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

// Tries a job has already had before the engine sees it (the retry list: the
// first pass ran one); the engine's give-up bound counts them.
template <class H>
__device__ __forceinline__ auto hb_resumed_tries(const H &, int) -> decltype(H::kResumedTries, u32()) {
    return H::kResumedTries;
}
template <class H>
__device__ __forceinline__ u32 hb_resumed_tries(const H &, long) { return 0u; }

template <int NL, int NR, class H, int MODE = 0>
__device__ __forceinline__ void hb_engine(H &h, const LaneTab &L, const PrfParams<NL> &P,
                                          u64 njobs, unsigned long long *queue, u64 chunk = HB_QUEUE_CHUNK) {
    HbPool pool{0, 0, njobs, queue, false, chunk};
    u64 job = 0;
    bool active = pool.take(__ballot(1), true, job);
    u32 dig[8], sr[4] = {0, 0, 0, 0}, out[NL];
    if (active) {
        h.init(job, sr);
        hb_job_digest<MODE>(h, job, dig, 0);
    }
    const u32 resumed = hb_resumed_tries(h, 0);
    u32 tries = 0, job_tries = resumed, failed = 0;
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
                job_tries = resumed;
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

// ------------------------------------------------------------------ quad PRF engine
// Latency-bound launches (a prove's 2 x 10,000 evaluations, verify, alpha,
// small KeyedPRF batches) last as long as their longest rejection chain: one
// lane runs nb serial CFB-8 steps per try, 14 dependent T-table rounds each,
// and a lone wave issues a round's 16 address v_perm + 16 ds_read_b32 + 8
// XORs back to back.  Here FOUR lanes run one evaluation: lane q = lane & 3
// holds column word q of the AES state and looks up T0..T3 of ITS column's
// four bytes; the XOR of a round's output column c = T0(lane c) ^ T1(lane c+1)
// ^ T2(lane c+2) ^ T3(lane c+3) ^ rk_c is gathered with DPP quad permutations.
// A round's serial chain drops from ~40 issued instructions to ~12.  Every
// lane of a quad computes the same keystream byte, ciphertext and output
// value, so the rejection test and the job queue stay quad-uniform.
#define HB_QP(a, b, c, d) ((a) | ((b) << 2) | ((c) << 4) | ((d) << 6))

template <int CTRL>
__device__ __forceinline__ u32 hb_qdpp(u32 x) {
    return (u32)__builtin_amdgcn_mov_dpp((int)x, CTRL, 0xf, 0xf, false);
}
__device__ __forceinline__ u64 hb_qbcast64(u64 v) {   // lane q = 0's value to its quad
    const u32 lo = hb_qdpp<HB_QP(0, 0, 0, 0)>((u32)v), hi = hb_qdpp<HB_QP(0, 0, 0, 0)>((u32)(v >> 32));
    return ((u64)hi << 32) | lo;
}

struct QuadLane {
    LaneTab L;
    u32 lbq;       // lane base of T_q
    u32 selq;      // v_perm selector: address of T_q[byte q of x]
    u32 sels;      // CFB shift: {next.0 | u.1, s.3, s.2, s.1}
    bool q3;       // the lane holding register bytes 12..15
};

__device__ __forceinline__ QuadLane hb_quad_lane(const LaneTab &L) {
    const u32 q = hb_lane_id() & 3u;
    QuadLane Q;
    Q.L = L;
    Q.lbq = q == 0 ? L.lb[0] : q == 1 ? L.lb[1] : q == 2 ? L.lb[2] : L.lb[3];
    Q.selq = 0x0c020000u | ((4u + q) << 8);
    Q.q3 = q == 3;
    Q.sels = Q.q3 ? 0x05030201u : 0x04030201u;
    return Q;
}

// One T-table round on the quad's column words (w = column q).
__device__ __forceinline__ u32 hb_quad_round(const LaneTab &L, u32 w, u32 rk) {
    const u32 a = hb_t<0, 0>(L, w), b = hb_t<1, 1>(L, w), c = hb_t<2, 2>(L, w), d = hb_t<3, 3>(L, w);
    const u32 x = hb_xor3(a, rk, hb_qdpp<HB_QP(1, 2, 3, 0)>(b));
    return hb_xor3(x, hb_qdpp<HB_QP(2, 3, 0, 1)>(c), hb_qdpp<HB_QP(3, 0, 1, 2)>(d));
}

// hb_cfb8_step for a quad: s = register column q, rkq[r] = rk[4r + q].
template <int NR>
__device__ __forceinline__ void hb_quad_cfb8_step(const QuadLane &Q, const u32 *rkq, const u32 *rk, u32 &s, u32 pk) {
    u32 w = s ^ rkq[0];
    HB_UNROLL
    for (int r = 1; r <= NR - 2; ++r) w = hb_quad_round(Q.L, w, rkq[r]);
    // byte 0 of round NR-1's column 0: lane q contributes T_q[byte q of column q]
    u32 x = hb_tab_ld(Q.L.tab, hb_perm(w, Q.lbq, Q.selq));
    x ^= hb_qdpp<HB_QP(1, 0, 3, 2)>(x);
    x = hb_xor3(x, hb_qdpp<HB_QP(2, 3, 0, 1)>(x), rk[4 * (NR - 1)]);
    const u32 u = hb_xor3(hb_t<0, 0>(Q.L, x), pk, rk[4 * NR] << 8);   // byte 1: the ciphertext byte
    const u32 nx = hb_qdpp<HB_QP(1, 2, 3, 0)>(s);
    s = hb_perm(Q.q3 ? u : nx, s, Q.sels);
}

// The newest four ciphertext bytes (register bytes 12..15, lane 3) as a
// big-endian word, on every lane of the quad.
__device__ __forceinline__ u32 hb_quad_s3_be(u32 s) { return hb_bswap(hb_qdpp<HB_QP(3, 3, 3, 3)>(s)); }

// hb_prf_try (FIRST = 0) for a quad.
template <int NL, int NR>
__device__ __forceinline__ u32 hb_quad_prf_try(const QuadLane &Q, const u32 *rkq, const PrfParams<NL> &P, u32 &s,
                                               const u32 dig[8], u32 out[NL]) {
    u32 dq[8];
    HB_UNROLL
    for (int t = 0; t < 8; ++t) dq[t] = dig[t];
    HB_UNROLL
    for (int t = 0; t < NL; ++t) out[t] = 0;
    const u32 nw = P.nb >> 2, tail = P.nb & 3u;
    u32 top = (P.topmask << 24) | 0xffffffu;
    HB_NOUNROLL
    for (u32 wi = 0; wi < nw; ++wi) {
        const u32 d = dq[0];
        hb_quad_cfb8_step<NR>(Q, rkq, P.rk, s, d >> 16);
        hb_quad_cfb8_step<NR>(Q, rkq, P.rk, s, d >> 8);
        hb_quad_cfb8_step<NR>(Q, rkq, P.rk, s, d);
        hb_quad_cfb8_step<NR>(Q, rkq, P.rk, s, d << 8);
        const u32 word = hb_quad_s3_be(s) & top;
        top = 0xffffffffu;
        HB_UNROLL
        for (int t = 0; t < 7; ++t) dq[t] = dq[t + 1];
        dq[7] = 0;
        HB_UNROLL
        for (int t = NL - 1; t > 0; --t) out[t] = out[t - 1];
        out[0] = word;
    }
    if (tail) {
        const u32 d = dq[0];
        for (u32 bi = 0; bi < tail; ++bi) hb_quad_cfb8_step<NR>(Q, rkq, P.rk, s, d >> (16 - 8 * bi));
        const u32 sh = 32 - 8 * tail;
        u32 word = hb_quad_s3_be(s) & (0xffffffffu >> sh);
        if (nw == 0) word &= (P.topmask << (24 - sh)) | (0xffffffu >> sh);
        HB_UNROLL
        for (int t = NL - 1; t > 0; --t) out[t] = hb_alignbit(out[t], out[t - 1], sh);
        out[0] = hb_alignbit(out[0], word << sh, sh);
    }
    u32 borrow = 0;
    HB_UNROLL
    for (int t = 0; t < NL; ++t) {
        u64 d = (u64)out[t] - (u64)P.R[t] - (u64)borrow;
        borrow = (u32)(d >> 63);
    }
    return borrow;
}

// hb_engine (MODE 0, fresh evaluations: h.init zeroes the register) with one
// job per quad.  Only lane q = 0 of a quad takes jobs and calls h.accept; the
// job index is broadcast to the quad.  `chunk` = jobs per refill per wave
// (16 = one per quad).  `first` != ~0: the wave runs jobs [first, min(first
// + 16, njobs, end)) and never touches the queue (placed waves,
// hb_prove_place).  A job abandoned after HB_MAX_TRIES is reported to
// h.fail (the fused prove's consumers wait for every job).
template <int NL, int NR, class H>
__device__ __forceinline__ void hb_engine_quad(H &h, const LaneTab &L, const PrfParams<NL> &P, u64 njobs,
                                               unsigned long long *queue, u64 chunk, u64 first = ~0ull,
                                               u64 end = ~0ull) {
    const QuadLane Q = hb_quad_lane(L);
    const u32 q = hb_lane_id() & 3u;
    const bool lead = q == 0;
    // rkq[r] = rk[4r + q]: select VALUES (readfirstlane: uniform SGPRs), not
    // addresses -- a lane-dependent index into the kernel argument struct
    // makes the compiler copy the whole struct to scratch
    u32 rkq[NR + 1];
    HB_UNROLL
    for (int r = 0; r <= NR; ++r) {
        const u32 k0 = __builtin_amdgcn_readfirstlane(P.rk[4 * r]), k1 = __builtin_amdgcn_readfirstlane(P.rk[4 * r + 1]);
        const u32 k2 = __builtin_amdgcn_readfirstlane(P.rk[4 * r + 2]), k3 = __builtin_amdgcn_readfirstlane(P.rk[4 * r + 3]);
        rkq[r] = q == 0 ? k0 : q == 1 ? k1 : q == 2 ? k2 : k3;
    }
    u64 stop = njobs - first < 16 ? njobs : first + 16;
    if (stop > end) stop = end;
    HbPool pool = first == ~0ull ? HbPool{0, 0, njobs, queue, false, chunk}
                                 : HbPool{first, stop, njobs, queue, true, chunk};
    u64 job = 0;
    bool active = pool.take(__ballot(lead), lead, job);
    job = hb_qbcast64(job);
    active = hb_qdpp<HB_QP(0, 0, 0, 0)>(active ? 1u : 0u) != 0;
    u32 dig[8], s = 0, out[NL];
    if (active) hb_job_digest<0>(h, job, dig, 0);
    u32 tries = 0, job_tries = 0, failed = 0;
    while (__ballot(active)) {
        const u32 ok = hb_quad_prf_try<NL, NR>(Q, rkq, P, s, dig, out);
        tries += active && lead ? 1u : 0u;
        job_tries += 1u;
        const bool acc = active && ok;
        if (acc && lead) h.accept(job, out);
        const bool give_up = active && !ok && job_tries >= HB_MAX_TRIES;
        failed += give_up && lead ? 1u : 0u;
        if (give_up && lead) h.fail(job);
        const bool next = acc || give_up;
        const u64 m = __ballot(next && lead);
        if (m) {
            u64 nj = 0;
            bool got = pool.take(m, next && lead, nj);
            nj = hb_qbcast64(nj);
            got = hb_qdpp<HB_QP(0, 0, 0, 0)>(got ? 1u : 0u) != 0;
            if (next) {
                active = got;
                job = nj;
                job_tries = 0;
                if (got) {
                    s = 0;   // fresh cipher per eval (util.py:88)
                    hb_job_digest<0>(h, job, dig, 0);
                }
            }
        }
    }
    for (int off = 32; off > 0; off >>= 1) {
        tries += __shfl_xor(tries, off);
        failed += __shfl_xor(failed, off);
    }
    if (hb_lane_id() == 0 && tries) atomicAdd(queue + 1, (unsigned long long)tries);
    if (hb_lane_id() == 0 && failed) atomicAdd(queue + 2, (unsigned long long)failed);
}

// The retry pass's engine (hb_encode_retry_kernel, 256-bit primes): hb_engine
// (MODE 0) while the job queue lasts; once it is drained and at most 16 lanes
// of the wave are still inside a rejection chain, each of those chains moves
// to a quad -- the r-th such lane's job, tries, digest and CFB-8 register
// (word q to lane q of quad r, the quad engine's layout) -- and finishes on
// the quad engine's round (hb_quad_prf_try: ~147 clocks per AES round against
// ~300 for a lone lane running all 16 lookups).  The pass ends on its longest
// chains, so this halves its tail.  The quads' accept runs the block's
// finish on one lane (the MFMA path's partial sum + F: cheap at NL = 8; the
// split wide-prime encode's F store, ALIGN = 0).  The wide primes need it
// most: a 1024-bit try is 128 serial AES, and the longest of ~3 M retry
// chains runs ~17 tries.
#ifndef HB_RETRY_QUAD_TAIL
#define HB_RETRY_QUAD_TAIL 1
#endif
template <int NL, int NR, class H>
__device__ __forceinline__ void hb_engine_tail(H &h, const LaneTab &L, const PrfParams<NL> &P, u64 njobs,
                                               unsigned long long *queue, u64 chunk) {
    HbPool pool{0, 0, njobs, queue, false, chunk};
    u64 job = 0;
    bool active = pool.take(__ballot(1), true, job);
    u32 dig[8], sr[4] = {0, 0, 0, 0}, out[NL];
    if (active) {
        h.init(job, sr);
        hb_job_digest<0>(h, job, dig, 0);
    }
    const u32 resumed = hb_resumed_tries(h, 0);
    u32 tries = 0, job_tries = resumed, failed = 0;
    u64 am;
    while ((am = __ballot(active)) != 0) {
        if (pool.exhausted && pool.next >= pool.end && __popcll(am) <= 16) break;   // -> quads
        const u32 ok = hb_prf_try<NL, NR>(L, P, sr, dig, out);
        tries += active ? 1u : 0u;
        job_tries += 1u;
        const bool acc = active && ok;
        if (acc) h.accept(job, out);
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
                job_tries = resumed;
                if (got) {
                    h.init(job, sr);
                    hb_job_digest<0>(h, job, dig, 0);
                }
            }
        }
    }
    if (am) {
        // quad r (lanes 4r .. 4r+3) takes the r-th lane of am
        const u32 lane = hb_lane_id(), r = lane >> 2, q = lane & 3u;
        const bool qa = r < (u32)__popcll(am);
        u64 mm = am;
        for (u32 k = 0; k < r && mm; ++k) mm &= mm - 1;
        const int src = mm ? __builtin_ctzll(mm) : 0;
        const u64 qjob = ((u64)(u32)__shfl((int)(u32)(job >> 32), src) << 32) | (u32)__shfl((int)(u32)job, src);
        u32 qdig[8];
        HB_UNROLL
        for (int t = 0; t < 8; ++t) qdig[t] = (u32)__shfl((int)dig[t], src);
        const u32 w0 = (u32)__shfl((int)sr[0], src), w1 = (u32)__shfl((int)sr[1], src);
        const u32 w2 = (u32)__shfl((int)sr[2], src), w3 = (u32)__shfl((int)sr[3], src);
        u32 s = q == 0 ? w0 : q == 1 ? w1 : q == 2 ? w2 : w3;
        u32 jt = (u32)__shfl((int)job_tries, src);
        const QuadLane Q = hb_quad_lane(L);
        u32 rkq[NR + 1];
        HB_UNROLL
        for (int rr = 0; rr <= NR; ++rr) {
            const u32 k0 = __builtin_amdgcn_readfirstlane(P.rk[4 * rr]), k1 = __builtin_amdgcn_readfirstlane(P.rk[4 * rr + 1]);
            const u32 k2 = __builtin_amdgcn_readfirstlane(P.rk[4 * rr + 2]), k3 = __builtin_amdgcn_readfirstlane(P.rk[4 * rr + 3]);
            rkq[rr] = q == 0 ? k0 : q == 1 ? k1 : q == 2 ? k2 : k3;
        }
        const bool lead = q == 0;
        bool qact = qa;
        u32 qtries = 0, qfailed = 0;
        while (__ballot(qact)) {
            const u32 ok = hb_quad_prf_try<NL, NR>(Q, rkq, P, s, qdig, out);
            qtries += qact && lead ? 1u : 0u;
            jt += 1u;
            if (qact && ok && lead) h.accept(qjob, out);
            const bool give_up = qact && !ok && jt >= HB_MAX_TRIES;
            qfailed += give_up && lead ? 1u : 0u;
            if (ok || give_up) qact = false;
        }
        tries += qtries;
        failed += qfailed;
    }
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
// Threads per workgroup of the encode kernels: 1,024 (16 waves sharing one
// LDS table image per CU), but 512 for primes above 512 bits, whose 2NL+1-limb
// MAC accumulator, REDC and PRF output do not fit the 128 VGPRs a lane of a
// 1,024-thread workgroup gets (NL = 32 spilled 576-656 B per lane): 256
// VGPRs, 8 waves per CU.
#ifndef HB_WIDE_WG
#define HB_WIDE_WG 512
#endif
// The F-only passes (ALIGN = 0) of 2048-bit primes hold a 64-limb PRF output
// per lane: under a 1,024-thread workgroup's 128 VGPRs they spilled 276 bytes
// per lane; 768 threads (12 waves per CU, 170 VGPRs) is the A/B candidate.
#ifndef HB_F64_WG
#define HB_F64_WG 768
#endif
#ifndef HB_WIDE_NL
#define HB_WIDE_NL 32
#endif
template <int NL>
struct HbEncodeWg { static constexpr int v = NL >= HB_WIDE_NL ? HB_WIDE_WG : HB_ENGINE_WG; };
// ALIGN = 0: the split wide-prime encode's PRF passes, which only store F
// (the MAC is hb_wmac_kernel's): no MAC accumulator, so 1,024-thread
// workgroups at every prime size -- 16 waves per CU on one LDS table image,
// the 256-bit kernel's occupancy
template <int NL, int ALIGN>
struct HbEncWg { static constexpr int v = ALIGN == 0 ? (NL >= 64 ? HB_F64_WG : HB_ENGINE_WG) : HbEncodeWg<NL>::v; };


__device__ __forceinline__ void hb_zero_sr(u32 sr[4]) { sr[0] = sr[1] = sr[2] = sr[3] = 0; }

// NL little-endian limbs to 16-byte aligned global memory (NL % 4 == 0)
template <int NL>
__device__ __forceinline__ void hb_store_limbs(u32 *dst, const u32 v[NL]) {
    HB_UNROLL
    for (int t = 0; t < NL; t += 4) *reinterpret_cast<uint4 *>(dst + t) = make_uint4(v[t], v[t + 1], v[t + 2], v[t + 3]);
}

template <int NL, int ALIGN, int MODE = 0>
struct EncodeHandler {
    const EncodeArgs<NL> &A;
    __device__ __forceinline__ u64 x_of(u64 job) const { return A.block_base + job; }
    __device__ __forceinline__ void init(u64, u32 sr[4]) const { hb_zero_sr(sr); }
    __device__ __forceinline__ void accept(u64 job, const u32 F[NL]) const {
        if constexpr (ALIGN == 0) {   // split wide-prime encode: F for hb_wmac_kernel
            if (MODE == 1 && job * A.C >= A.len) {
                // cxx, no sector read: the tag is F itself, unreduced
                // (shacham_waters_private.cxx:681-690); no MAC kernel reads it
                hb_store_be<NL>(A.tags + job * (u64)A.tw, A.tw, F);
                return;
            }
            hb_store_limbs<NL>(A.fout + job * NL, F);
        } else {
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
            hb_store_tag<NL, ALIGN>(A.tags + job * (u64)A.tw, A.tw, tag);
#endif
        }
    }
};

template <int NL, int NR, int ALIGN>
__global__ __launch_bounds__((HbEncWg<NL, ALIGN>::v), HbEncodeOcc<NL>::v) void hb_encode_kernel(EncodeArgs<NL> A) {
    __shared__ __attribute__((aligned(16))) u32 lds[HB_LDS_WORDS];
    hb_fill_lds(lds, A.t0);
    const LaneTab L = hb_lane_tab(lds);
    EncodeHandler<NL, ALIGN> h{A};
    hb_engine<NL, NR>(h, L, A.prf, A.nblocks, A.queue, hb_qchunk(A.qchunk));
}

// Small inputs (hb_runtime.cpp: as many blocks as the quad engine runs at
// once): the two-pass engine's fixed costs -- the 2^24-entry prefix image and
// a retry pass whose lone lanes each run a whole 14-round AES per CFB-8 step
// -- outweigh its throughput, so F(block_base + k) comes from one quad-engine
// PRF launch (four lanes per evaluation, every try in one chain) and this
// kernel adds the sector MAC, one lane per block: tag = F + sum_j alpha_j
// m_kj mod p (hb_block_tag, the single-pass encode's MAC; PySwizzle.py:297-307).
template <int NL, int ALIGN>
__global__ __launch_bounds__(256) void hb_mac_kernel(EncodeArgs<NL> A) {
    const u64 k = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= A.nblocks) return;
    u32 F[NL], tag[NL];
    for (int t = 0; t < NL; ++t) F[t] = A.fv[k * NL + t];
    hb_block_tag<NL, ALIGN>(A.data, A.len, k, A.C, A.ss, A.S, A.alpha_mont, A.mod, F, tag);
    hb_store_tag<NL, ALIGN>(A.tags + k * (u64)A.tw, A.tw, tag);
}

// hb_mac_kernel with the sectors of a block spread over S lanes (S <= T): lane
// (k, j) forms alpha_j R * m_kj (+ F_k R on lane j = 0) and reduces it
// (REDC: alpha_j m_kj [+ F_k] mod p), and lane (k, 0) adds the S residues mod
// p.  A small input has too few blocks to fill the GPU with one lane each
// (820 at PySwizzle's defaults on 1 MiB: four workgroups, every lane a serial
// chain of S x NL^2 multiply-adds); this cuts the chain to NL^2 + REDC.
// Sector values as hb_block_tag's: BE(data[off, min(off + ss, len))), 0 past
// the end of the file.
template <int NL>
struct HbMacSplit { static constexpr int T = NL >= 64 ? 128 : 256; };
template <int NL, int ALIGN>
__global__ __launch_bounds__(HbMacSplit<NL>::T) void hb_mac_split_kernel(EncodeArgs<NL> A) {
    constexpr int T = HbMacSplit<NL>::T;
    __shared__ u32 red[T * NL];
    const u32 S = A.S, bpw = T / S;
    const u32 lb = threadIdx.x / S, j = threadIdx.x % S;
    const u64 k = (u64)blockIdx.x * bpw + lb;
    const bool live = lb < bpw && k < A.nblocks;
    if (live) {
        u32 acc[2 * NL + 1], m[NL];
        for (int t = 0; t <= 2 * NL; ++t) acc[t] = 0;
        if (j == 0)
            for (int t = 0; t < NL; ++t) acc[NL + t] = A.fv[k * NL + t];
        const u64 off = k * A.C + (u64)j * A.ss;
        if (off < A.len) {
            const u32 r = (u32)(A.len - off < A.ss ? A.len - off : A.ss);
            if (ALIGN == 16 && r == A.ss) hb_load_full16<NL>(A.data, off, m);
            else hb_load_be_bytes<NL>(A.data, off, r, m);
            hb_mac<NL>(acc, A.alpha_mont + (u64)j * NL, m);
        }
        u32 v[NL + 1], res[NL];
        hb_redc<NL>(acc, A.mod, v);
        hb_reduce_small<NL>(v, A.mod, res);
        for (int t = 0; t < NL; ++t) red[threadIdx.x * NL + t] = res[t];
    }
    __syncthreads();
    if (!live || j != 0) return;
    u32 v[NL + 1], tag[NL];
    u64 c = 0;
    for (int t = 0; t < NL; ++t) {   // S residues < p: the sum < S p < 2^32 p
        c += red[threadIdx.x * NL + t];
        for (u32 i = 1; i < S; ++i) c += red[(threadIdx.x + i) * NL + t];
        v[t] = (u32)c;
        c >>= 32;
    }
    v[NL] = (u32)c;
    hb_reduce_small<NL>(v, A.mod, tag);
    hb_store_tag<NL, ALIGN>(A.tags + k * (u64)A.tw, A.tw, tag);
}

// The cxx Swizzle encode (shacham_waters_private.cxx:638-702): the same
// engine and MAC with the cxx prf (CFB-128: nb/16 full AES per try instead of
// nb byte-0 AES).
template <int NL, int NR, int ALIGN>
__global__ __launch_bounds__((HbEncWg<NL, ALIGN>::v), HbEncodeOcc<NL>::v) void hb_cxx_encode_kernel(EncodeArgs<NL> A) {
    __shared__ __attribute__((aligned(16))) u32 lds[HB_LDS_WORDS];
    hb_fill_lds(lds, A.t0);
    const LaneTab L = hb_lane_tab(lds);
    EncodeHandler<NL, ALIGN, 1> h{A};
    hb_engine<NL, NR, EncodeHandler<NL, ALIGN, 1>, 1>(h, L, A.prf, A.nblocks, A.queue, hb_qchunk(A.qchunk));
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

// ------------------------------------------------------------------ MFMA MAC
// sum_j (alpha_j R mod p) m_ij for the 64 blocks of a wave (one per lane) on
// the matrix cores, for 256-bit primes (ss = 32 = 4 NL, aligned sectors).
// With alpha'_j = sum_d a_jd 256^d in signed digits a_jd in [-128, 127]
// (33 digits) and the sector bytes entering as u - 128:
//     sum_j alpha'_j m_ij = Q sum_j alpha'_j + sum_c D_ic 256^c,
//     D_ic = sum_j sum_b (u_ijb - 128) a_{j, c-31+b},   c < 64
// (byte b of a sector has weight 256^(31-b)), i.e. for every sector j one
// v_mfma_i32_32x32x32_i8 per 32 blocks and 32 output columns: A = the digit
// Toeplitz matrix of sector j (32 columns c x 32 bytes b, host-built
// fragments), B = the 32 bytes of sector j of 32 blocks (one 16-byte load per
// lane).  |D_ic| <= S 32 2^14 < 2^31.  Lanes 0-31 feed blocks of lanes 0-31
// (group 0), lanes 32-63 ... (group 1); lane half h of a 32x32 result holds
// the 32-bit limbs 2k + h of its column's block (rows 8q + 4h + r: byte r of
// limb 8t + 2q + h), so one exchange with lane l ^ 32 gives every lane all
// 16 limbs of its OWN block.  The lane then forms
//     T = kz + sum_t L_t 2^(32 t)     (kz = Q sum_j alpha'_j mod p + p 2^268 > 0)
// with T == sum_j alpha'_j m_ij (mod p), 0 < T < 2^544: the Montgomery
// accumulator of hb_block_tag without F R, off the VALU.
typedef int32_t hb_i32x4 __attribute__((ext_vector_type(4)));
typedef int32_t hb_i32x16 __attribute__((ext_vector_type(16)));

template <int NL>
__device__ __forceinline__ bool hb_block_full(const EncodeArgs<NL> &A, u64 job) {
    return (job + 1) * A.C <= A.len;
}

// Wave-uniform call.  Returns whether THIS lane's T is valid (active lane,
// block entirely inside the data); T has 2NL+1 = 17 limbs.  Lane half g
// (lanes 32g .. 32g+31) owns group g's blocks.  Per sector ONE MFMA with the
// dense A tile of the reduced digits (hb_runtime.cpp, mfma_tables) gives the
// 32 output digits of the group's blocks, i.e. 8 signed 64-bit limbs (with
// HB_MFMA_TOEPLITZ two MFMAs, 64 digits, 16 limbs).  After both groups every
// lane holds, per group, the limbs 2k + h (h = its half) of the group's
// column-n block; one v_permlane32_swap per dword (lanes 32-63 of the first
// operand <-> lanes 0-31 of the second, with G0 first and G1 second) then
// leaves every lane with the EVEN limbs of its own block in the first result
// and the ODD limbs in the second, and T is assembled once, by all lanes.
// The sector loads of a group go out HB_MFMA_BATCH at a time before their
// MFMAs (one memory latency per batch, not per sector); the A fragments come
// from LDS (`afl`, S <= HB_MFMA_LDS_S) or global memory.
#ifndef HB_MFMA_BATCH
#define HB_MFMA_BATCH 4
#endif
#define HB_MFMA_LDS_S 16
// issue priority of a first try's AES (s_setprio; the rest of the loop runs at 0)
#ifndef HB_AES_PRIO
#define HB_AES_PRIO 2
#endif

// x of lane (l ^ 1) / (l ^ 2) within the lane's quad (DPP quad_perm)
__device__ __forceinline__ int32_t hb_quad_x1(int32_t x) { return __builtin_amdgcn_mov_dpp(x, 0xB1, 0xf, 0xf, false); }
__device__ __forceinline__ int32_t hb_quad_x2(int32_t x) { return __builtin_amdgcn_mov_dpp(x, 0x4E, 0xf, 0xf, false); }

// Whole-line sector loads for the MFMA MAC (EncodeArgs::mfma == 2, S % 4 == 0):
// the 4 sectors j0 .. j0+3 of the 32 blocks of group g, i.e. one 128-byte line
// per block, as 4 loads in which each lane quad reads one contiguous 64-byte
// half line (lane (h, 4q + i) of load r: chunk 4h + i of block 4q + r), so
// every line is requested by ONE instruction in whole 64-byte pieces (the
// sector-shaped loads request each line from 4 instructions, 16 bytes a lane:
// measured 3.1x the L1 accesses and 1.13x the L1 -> L2 requests; worth
// +0.3 %).  A 4 x 4
// transpose inside each quad (lane bits 0-1 <-> load index, two DPP exchange
// stages) then leaves in V[r'] at lane (h, n) chunk 4h + r' of block n: the
// MFMA B layout, with the A fragments of slot j0 + r' built for those chunks
// (hb_runtime.cpp, mfma_tables).
__device__ __forceinline__ void hb_line_loads(const unsigned char *const blk[4], const bool okr[4], u32 off,
                                              hb_i32x4 V[4]) {
    hb_i32x4 L[4];
#pragma unroll
    for (int r = 0; r < 4; ++r)
        L[r] = okr[r] ? *reinterpret_cast<const hb_i32x4 *>(blk[r] + off) : hb_i32x4{0, 0, 0, 0};
    const u32 i = hb_lane_id() & 3u;
    const bool b0 = i & 1u, b1 = i & 2u;
    hb_i32x4 M[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
        // stage 1: M_{r1 r0}[i1 i0] = L_{r1 i0}[i1 r0]
        const int32_t x0 = hb_quad_x1(L[0][e]), x1 = hb_quad_x1(L[1][e]);
        const int32_t x2 = hb_quad_x1(L[2][e]), x3 = hb_quad_x1(L[3][e]);
        M[0][e] = b0 ? x1 : L[0][e];
        M[1][e] = b0 ? L[1][e] : x0;
        M[2][e] = b0 ? x3 : L[2][e];
        M[3][e] = b0 ? L[3][e] : x2;
    }
#pragma unroll
    for (int e = 0; e < 4; ++e) {
        // stage 2: V_{r1 r0}[i1 i0] = M_{i1 r0}[r1 i0] = L_{i1 i0}[r1 r0]
        const int32_t y0 = hb_quad_x2(M[0][e]), y1 = hb_quad_x2(M[1][e]);
        const int32_t y2 = hb_quad_x2(M[2][e]), y3 = hb_quad_x2(M[3][e]);
        V[0][e] = b1 ? y2 : M[0][e];
        V[2][e] = b1 ? M[2][e] : y0;
        V[1][e] = b1 ? y3 : M[1][e];
        V[3][e] = b1 ? M[3][e] : y1;
    }
}

template <int NL, bool ALDS>
__device__ __forceinline__ bool hb_mfma_block_acc(const EncodeArgs<NL> &A, const hb_i32x4 *afl, u64 job, bool active,
                                                  u32 T[2 * NL + 1]) {
    static_assert(NL == 8, "MFMA MAC: 256-bit primes only");
    const u32 l = hb_lane_id(), h = l >> 5, n = l & 31u;
    const bool mine = active && hb_block_full(A, job);
    const u32 S = A.S;
    constexpr int NK = 4 * HB_MFMA_NT;   // limbs per lane half and group
    long long G[2][NK];   // G[g][k]: limb 2k + h of group g's column-n block
#pragma unroll
    for (u32 g = 0; g < 2; ++g) {
        hb_i32x16 acc0 = {};
#if defined(HB_MFMA_TOEPLITZ)
        hb_i32x16 acc1 = {};
#endif
#if !defined(HB_NO_LINE_LOADS)
        if (A.mfma == 2) {
            // load r of lane (h, 4q + i) reads block 4q + r of the group (lane 32 g + 4q + r's)
            const unsigned char *blk[4];
            bool okr[4];
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int src = (int)(32 * g + (n & ~3u) + r);
                const u64 jb = (u64)__shfl((long long)job, src);
                okr[r] = __shfl((int)mine, src) != 0;
                blk[r] = A.data + jb * A.C + 64u * h + 16u * (l & 3u);
            }
            for (u32 j0 = 0; j0 < S; j0 += 4) {
                hb_i32x4 V[4];
                hb_line_loads(blk, okr, 32u * j0, V);
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const hb_i32x4 bb = V[r] ^ (int32_t)0x80808080;
                    acc0 = __builtin_amdgcn_mfma_i32_32x32x32_i8(afl[(j0 + r) * 64 + l], bb, acc0, 0, 0, 0);
#if defined(HB_MFMA_TOEPLITZ)
                    acc1 = __builtin_amdgcn_mfma_i32_32x32x32_i8(afl[(S + j0 + r) * 64 + l], bb, acc1, 0, 0, 0);
#endif
                }
            }
        } else
#endif
        {
        // the block of column n in group g: lane 32 g + n's
        const u64 jb = (u64)__shfl((long long)job, (int)(32 * g + n));
        const bool ok = __shfl((int)mine, (int)(32 * g + n)) != 0;
        const hb_i32x4 *src = reinterpret_cast<const hb_i32x4 *>(A.data + jb * A.C + 16u * h);
        for (u32 j0 = 0; j0 < S; j0 += HB_MFMA_BATCH) {
            hb_i32x4 b[HB_MFMA_BATCH];
#pragma unroll
            for (int jj = 0; jj < HB_MFMA_BATCH; ++jj)
#if defined(HB_EXP_MFMA_NOLOAD)   // phase-cost experiment only (wrong tags): no sector loads
                (void)ok; (void)src;
                b[jj] = hb_i32x4{(int32_t)jb, (int32_t)(j0 + jj), 1, 2};
#else
                b[jj] = ok && j0 + jj < S ? src[2 * (j0 + jj)] : hb_i32x4{0, 0, 0, 0};
#endif
#pragma unroll
            for (int jj = 0; jj < HB_MFMA_BATCH; ++jj) {
                // past the last sector: a zero B (after the -128 shift) against
                // the last sector's A adds nothing
                const bool in = j0 + jj < S;
                const u32 j = in ? j0 + jj : S - 1;
                const hb_i32x4 bb = in ? b[jj] ^ (int32_t)0x80808080 : hb_i32x4{0, 0, 0, 0};
                acc0 = __builtin_amdgcn_mfma_i32_32x32x32_i8(afl[j * 64 + l], bb, acc0, 0, 0, 0);
#if defined(HB_MFMA_TOEPLITZ)
                acc1 = __builtin_amdgcn_mfma_i32_32x32x32_i8(afl[(S + j) * 64 + l], bb, acc1, 0, 0, 0);
#endif
            }
        }
        }
        // limb 8t + 2q + h of column n's block = bytes acc_t[4q .. 4q+3];
        // k = 4t + q: limb 2k + h
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            G[g][q] = (long long)acc0[4 * q] + ((long long)acc0[4 * q + 1] << 8) +
                      ((long long)acc0[4 * q + 2] << 16) + ((long long)acc0[4 * q + 3] << 24);
#if defined(HB_MFMA_TOEPLITZ)
            G[g][4 + q] = (long long)acc1[4 * q] + ((long long)acc1[4 * q + 1] << 8) +
                          ((long long)acc1[4 * q + 2] << 16) + ((long long)acc1[4 * q + 3] << 24);
#endif
        }
    }
    long long ev[NK], od[NK];   // limbs 2k and 2k + 1 of this lane's own block
#pragma unroll
    for (int k = 0; k < NK; ++k) {
        const auto lo = __builtin_amdgcn_permlane32_swap((int)(u32)G[0][k], (int)(u32)G[1][k], false, false);
        const auto hi = __builtin_amdgcn_permlane32_swap((int)(G[0][k] >> 32), (int)(G[1][k] >> 32), false, false);
        ev[k] = (long long)(((u64)(u32)hi[0] << 32) | (u32)lo[0]);
        od[k] = (long long)(((u64)(u32)hi[1] << 32) | (u32)lo[1]);
    }
    // T = kz + sum_t L_t 2^(32 t), signed carries
    long long carry = 0;
#pragma unroll
    for (int t = 0; t <= 2 * NL; ++t) {
        long long x = (long long)A.kz[t] + carry;
        if (t < 2 * NK) x += (t & 1) ? od[t >> 1] : ev[t >> 1];
        T[t] = (u32)x;
        carry = x >> 32;
    }
    return mine;
}

// The MAC on v_mfma_i32_16x16x64_i8 (EncodeArgs::mfma == 3, dense tiles,
// S % 2 == 0).  Its B operand is exactly the whole-line load shape: lane
// (q, n) = (l >> 4, l & 15) holds bytes 16 q .. 16 q + 15 of column n's
// 64-byte K slice, so for sectors 2p, 2p+1 the four lanes n, n+16, n+32, n+48
// read one contiguous 64-byte half line of block n: every load instruction
// requests 16 whole 64-byte pieces and no lane exchange is needed before the
// MFMA (the 32x32x32 line path, hb_line_loads, spends 2 x 16 DPP moves and
// selects per 4 sectors on that).  Group g (g < 4) is the 16 blocks of lanes
// 16 g .. 16 g + 15; two 16-row tiles (output digits 0-15, 16-31) per K
// slice, their A fragments read once per slice for all four groups.
// Afterwards lane (q, n) holds, per group g, limbs q and 4 + q of block
// 16 g + n; a 4 x 4 transpose of (group, lane row) -- one v_permlane32_swap
// stage and one v_permlane16_swap stage per dword -- leaves every lane with
// the 8 limbs of its own block.
template <int NL, bool ALDS>
__device__ __forceinline__ bool hb_mfma16_block_acc(const EncodeArgs<NL> &A, const hb_i32x4 *afl, u64 job,
                                                    bool active, u32 T[2 * NL + 1]) {
    static_assert(NL == 8, "MFMA MAC: 256-bit primes only");
    const u32 l = hb_lane_id(), q = l >> 4, n = l & 15u;
    const bool mine = active && hb_block_full(A, job);
    const u32 np = A.S / 2;   // K slices of 64 bytes (2 sectors)
    const unsigned char *blk[4];
    bool okg[4];
#pragma unroll
    for (int g = 0; g < 4; ++g) {
        const int src = (int)(16 * g + n);
        const u64 jb = (u64)__shfl((long long)job, src);
        okg[g] = __shfl((int)mine, src) != 0;
        blk[g] = A.data + jb * A.C + 16u * q;
    }
    hb_i32x4 acc[4][2];
#pragma unroll
    for (int g = 0; g < 4; ++g) acc[g][0] = acc[g][1] = hb_i32x4{0, 0, 0, 0};
    auto slice = [&](const hb_i32x4 b[4], u32 p) {
        const hb_i32x4 a0 = afl[(2 * p) * 64 + l], a1 = afl[(2 * p + 1) * 64 + l];
#pragma unroll
        for (int g = 0; g < 4; ++g) {
            const hb_i32x4 bb = b[g] ^ (int32_t)0x80808080;
            acc[g][0] = __builtin_amdgcn_mfma_i32_16x16x64_i8(a0, bb, acc[g][0], 0, 0, 0);
            acc[g][1] = __builtin_amdgcn_mfma_i32_16x16x64_i8(a1, bb, acc[g][1], 0, 0, 0);
        }
    };
    u32 p = 0;
    // two slices (one 128-byte line of every block) per round of loads
    for (; p + 1 < np; p += 2) {
        hb_i32x4 b0[4], b1[4];
#pragma unroll
        for (int g = 0; g < 4; ++g) {
            b0[g] = okg[g] ? *reinterpret_cast<const hb_i32x4 *>(blk[g] + 64u * p) : hb_i32x4{0, 0, 0, 0};
            b1[g] = okg[g] ? *reinterpret_cast<const hb_i32x4 *>(blk[g] + 64u * (p + 1)) : hb_i32x4{0, 0, 0, 0};
        }
        slice(b0, p);
        slice(b1, p + 1);
    }
    if (p < np) {
        hb_i32x4 b0[4];
#pragma unroll
        for (int g = 0; g < 4; ++g)
            b0[g] = okg[g] ? *reinterpret_cast<const hb_i32x4 *>(blk[g] + 64u * p) : hb_i32x4{0, 0, 0, 0};
        slice(b0, p);
    }
    // X[g][d]: dwords of limbs q (d = 0, 1) and 4 + q (d = 2, 3) of block 16 g + n
    u32 X[4][4];
#pragma unroll
    for (int g = 0; g < 4; ++g)
#pragma unroll
        for (int t = 0; t < 2; ++t) {
            const hb_i32x4 &a = acc[g][t];
            const long long v = (long long)a[0] + ((long long)a[1] << 8) + ((long long)a[2] << 16) +
                                ((long long)a[3] << 24);
            X[g][2 * t] = (u32)v;
            X[g][2 * t + 1] = (u32)((u64)v >> 32);
        }
#pragma unroll
    for (int d = 0; d < 4; ++d) {
        const auto s02 = __builtin_amdgcn_permlane32_swap((int)X[0][d], (int)X[2][d], false, false);
        const auto s13 = __builtin_amdgcn_permlane32_swap((int)X[1][d], (int)X[3][d], false, false);
        const auto s01 = __builtin_amdgcn_permlane16_swap((int)s02[0], (int)s13[0], false, false);
        const auto s23 = __builtin_amdgcn_permlane16_swap((int)s02[1], (int)s13[1], false, false);
        X[0][d] = (u32)s01[0];
        X[1][d] = (u32)s01[1];
        X[2][d] = (u32)s23[0];
        X[3][d] = (u32)s23[1];
    }
    // slot s: limbs s and 4 + s of this lane's block.  T = kz + sum_t L_t 2^(32 t)
    long long carry = 0;
#pragma unroll
    for (int t = 0; t <= 2 * NL; ++t) {
        long long x = (long long)A.kz[t] + carry;
        if (t < 8) {
            const int sl = t & 3, hi = t >> 2;
            x += (long long)(((u64)X[sl][2 * hi + 1] << 32) | X[sl][2 * hi]);
        }
        T[t] = (u32)x;
        carry = x >> 32;
    }
    return mine;
}

#if defined(HB_MAC_MONT)
// tag = (T + F R) R^-1 mod p  (T from hb_mfma_block_acc; F < 2^256 at limbs NL..)
template <int NL>
__device__ __forceinline__ void hb_finish_T(u32 T[2 * NL + 1], const u32 F[NL], const ModP<NL> &M, u32 out[NL]) {
    u64 c = 0;
    for (int t = 0; t < NL; ++t) {
        c += (u64)T[NL + t] + F[t];
        T[NL + t] = (u32)c;
        c >>= 32;
    }
    T[2 * NL] += (u32)c;
    u32 v[NL + 1];
    hb_redc<NL>(T, M, v);
    hb_reduce_small<NL>(v, M, out);
}
#else
// tag = (T + F) mod p: T (from hb_mfma_block_acc) = sum_j alpha_j m_j mod p
// plus a multiple of p, < 2^282 (hb_runtime.cpp, mfma_tables), so T + F fits
// NL + 1 limbs with a quotient below 2^27 -- one quotient-estimate reduction
// (hb_reduce_small), no Montgomery REDC
template <int NL>
__device__ __forceinline__ void hb_finish_T(u32 T[2 * NL + 1], const u32 F[NL], const ModP<NL> &M, u32 out[NL]) {
    u32 v[NL + 1];
    u64 c = 0;
    HB_UNROLL
    for (int t = 0; t < NL; ++t) {
        c += (u64)T[t] + F[t];
        v[t] = (u32)c;
        c >>= 32;
    }
    v[NL] = T[NL] + (u32)c;
    hb_reduce_small<NL>(v, M, out);
}
#endif

// End of the first try of every lane's block (wave-uniform call): accepted
// blocks are tagged, rejected ones go to the retry list with their shift
// register (and, with the MFMA MAC, with sum_j alpha_j m_j mod p, so that the
// retry pass only adds F).  With the MFMA MAC both cases are ONE reduction,
// (T + F') mod p with F' = F (accepted) or 0 (rejected) (hb_finish_T): with ~14 %
// rejected first tries nearly every wave has lanes of both kinds, and two
// divergent reductions would cost both per wave.
// HB_RETRY_DIGEST: list the lanes of `mask` (first output word above R's top
// word: rejected whatever the try's other bytes are) with their digest, before
// the try; `base` = the wave's first slot.
template <int NL>
__device__ __forceinline__ void hb_list_early(const EncodeArgs<NL> &A, u64 job, u64 mask, const u32 dig[8],
                                              u64 &base) {
#if HB_RETRY_DIGEST
    u64 b = 0;
    if (hb_lane_id() == 0) b = atomicAdd(A.retry_count, (unsigned long long)__popcll(mask));
    base = hb_bcast64(b);
    if ((mask >> hb_lane_id()) & 1ull) {
        const u64 slot = base + hb_mbcnt(mask);
        if (slot < A.retry_cap) {
            HbRetry *e = A.retry + slot;
            *reinterpret_cast<uint4 *>(e) = make_uint4((u32)job, (u32)(job >> 32), 1u, 0u);
            *reinterpret_cast<uint4 *>(e->dig) = make_uint4(dig[0], dig[1], dig[2], dig[3]);
            *reinterpret_cast<uint4 *>(e->dig + 4) = make_uint4(dig[4], dig[5], dig[6], dig[7]);
        }
    }
#endif
}

template <int NL, int NR, int ALIGN, class H>
__device__ __forceinline__ void hb_first_finish(const EncodeArgs<NL> &A, const LaneTab &L, H &h, u64 job,
                                                bool active, u32 ok, u32 sr[4], u32 out[NL], u32 &tries,
                                                u32 &failed, u32 *T, bool tmine, u64 pre_base, u64 pre_mask) {
    tries += active ? 1u : 0u;
    const bool rejected = active && !ok;
    // listed before the try (hb_list_early; always rejected)
    const bool pre = (pre_mask >> hb_lane_id()) & 1ull;
    const u64 rej = __ballot(rejected && !pre);
    bool listed = false;
    HbRetry *e = nullptr;
    if (pre) {
        const u64 slot = pre_base + hb_mbcnt(pre_mask);
        if (slot < A.retry_cap) {
            listed = true;
            e = A.retry + slot;
        }
    }
    if (rej) {
        u64 base = 0;
        if (hb_lane_id() == 0) base = atomicAdd(A.retry_count, (unsigned long long)__popcll(rej));
        base = hb_bcast64(base);
        if (rejected && !pre) {
            const u64 slot = base + hb_mbcnt(rej);
            if (slot < A.retry_cap) {
                listed = true;
                e = A.retry + slot;
                // no digest stored (flags 0): the retry pass hashes the index
                *reinterpret_cast<uint4 *>(e) = make_uint4((u32)job, (u32)(job >> 32), 0u, 0u);
            }
        }
    }
    if (listed) {
        *reinterpret_cast<uint4 *>(e->sr) = make_uint4(sr[0], sr[1], sr[2], sr[3]);
    } else if (rejected) {
        // retry list full (never at its sizing, see hb_runtime.cpp): finish
        // this eval in place
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
    const bool done = active && ok;
#if defined(HB_EXP_NO_FINISH)   // instruction-count experiment only (wrong tags)
    if (done) hb_store_be<NL>(A.tags + job * (u64)A.tw, A.tw, T + 3);
    return;
#endif
    if constexpr (NL == 8) {
        if (A.mfma) {
            if (tmine && (done || listed)) {
                u32 F[NL], res[NL];
                HB_UNROLL
                for (int t = 0; t < NL; ++t) F[t] = done ? out[t] : 0u;
                hb_finish_T<NL>(T, F, A.mod, res);
                if (done) {
                    hb_store_tag<NL, ALIGN>(A.tags + job * (u64)A.tw, A.tw, res);
                } else {
                    *reinterpret_cast<uint4 *>(e->part) = make_uint4(res[0], res[1], res[2], res[3]);
                    *reinterpret_cast<uint4 *>(e->part + 4) = make_uint4(res[4], res[5], res[6], res[7]);
                }
                return;
            }
            if (listed) {
                // a block the MFMA MAC does not cover (the short last block)
                const u32 zero[NL] = {0, 0, 0, 0, 0, 0, 0, 0};
                u32 part[NL];
                hb_block_tag<NL, ALIGN>(A.data, A.len, job, A.C, A.ss, A.S, A.alpha_mont, A.mod, zero, part);
                *reinterpret_cast<uint4 *>(e->part) = make_uint4(part[0], part[1], part[2], part[3]);
                *reinterpret_cast<uint4 *>(e->part + 4) = make_uint4(part[4], part[5], part[6], part[7]);
                return;
            }
        }
    }
    if (done) h.accept(job, out);
}

template <int NL, int NR, int ALIGN>
__global__ __launch_bounds__((HbEncWg<NL, ALIGN>::v), HbEncodeOcc<NL>::v) void hb_encode_first_kernel(EncodeArgs<NL> A) {
    // MFMA MAC for 256-bit primes with aligned full-width sectors (A.mfma set by the host)
    constexpr bool MF = NL == 8 && ALIGN == 16;
    // MF: the T-table image plus the MFMA A fragments (HB_MFMA_NT x S x 1 KiB,
    // S <= 16): 144 KiB (160 with HB_MFMA_TOEPLITZ), one workgroup per CU
    constexpr u32 AFW = MF ? HB_MFMA_NT * HB_MFMA_LDS_S * 64u * 4u : 0u;
    __shared__ __attribute__((aligned(16))) u32 lds[HB_LDS_WORDS + AFW];
    const bool alds = MF && A.mfma && A.S <= HB_MFMA_LDS_S;
    if (alds) {
        const uint4 *src = reinterpret_cast<const uint4 *>(A.afrag);
        uint4 *dst = reinterpret_cast<uint4 *>(lds + HB_LDS_WORDS);
        for (u32 k = threadIdx.x; k < HB_MFMA_NT * A.S * 64u; k += blockDim.x) dst[k] = src[k];
    }
    hb_fill_lds(lds, A.t0);
    const LaneTab L = hb_lane_tab(lds);
    EncodeHandler<NL, ALIGN> h{A};
    HbPool pool{0, 0, A.nblocks, A.queue, false, hb_qchunk(A.qchunk)};
    u32 tries = 0, failed = 0;
    for (;;) {
        u64 job = 0;
        const bool act = pool.take(__ballot(1), true, job);
        if (!__ballot(act)) break;
        u32 T[2 * NL + 1];
        bool tmine = false;
#if defined(HB_EXP_NO_MFMA)   // instruction-count experiment only (wrong tags)
        for (int t = 0; t <= 2 * NL; ++t) T[t] = (u32)job + t;
        tmine = act && hb_block_full(A, job);
        if (0)
#endif
        if constexpr (MF) {
            // two call sites, so that each sees which memory its A fragments
            // are in (LDS: ds_read_b128; global: global_load_dwordx4)
            const hb_i32x4 *afl_lds = reinterpret_cast<const hb_i32x4 *>(lds + HB_LDS_WORDS);
            const hb_i32x4 *afl_glb = reinterpret_cast<const hb_i32x4 *>(A.afrag);
#if !defined(HB_MFMA_TOEPLITZ)
            if (A.mfma == 3) {
                if (alds) tmine = hb_mfma16_block_acc<NL, true>(A, afl_lds, job, act, T);
                else tmine = hb_mfma16_block_acc<NL, false>(A, afl_glb, job, act, T);
            } else
#endif
            if (alds) tmine = hb_mfma_block_acc<NL, true>(A, afl_lds, job, act, T);
            else if (A.mfma) tmine = hb_mfma_block_acc<NL, false>(A, afl_glb, job, act, T);
        }
        u32 out[NL], sr[4], ok;
        u64 pre_base = 0, pre_mask = 0;
        {
            u32 dig[8];
            hb_sha256_decimal(A.block_base + job, dig);
            hb_prf_prefix<NL>(A.pfx, A.o0, A.prf, dig[0], sr, out);
#if HB_RETRY_DIGEST
            // the first output word alone decides all but ~2^-32 of the
            // rejections: list those evals now, while their digest is live
            pre_mask = __ballot(act && out[0] > A.rtop);
            if (pre_mask) hb_list_early<NL>(A, job, pre_mask, dig, pre_base);
#endif
            // waves in their AES phase go first in issue arbitration, so the
            // LDS stays fed while other waves hash or run the MAC (+0.8 %,
            // same-box A/B, profiles/r02/s13)
            __builtin_amdgcn_s_setprio(HB_AES_PRIO);
            ok = hb_prf_try_from<NL, NR, 1>(L, A.prf, sr, dig, out);
            __builtin_amdgcn_s_setprio(0);
        }
        hb_first_finish<NL, NR, ALIGN>(A, L, h, job, act, ok, sr, out, tries, failed, T, tmine, pre_base,
                                       pre_mask);
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
    static constexpr u32 kResumedTries = 1;   // the first pass ran one try
    const EncodeArgs<NL> &A;
    __device__ __forceinline__ u64 x_of(u64 job) const { return A.block_base + A.retry[job].blk; }
    __device__ __forceinline__ void init(u64 job, u32 sr[4]) const {
        const uint4 v = *reinterpret_cast<const uint4 *>(A.retry[job].sr);
        sr[0] = v.x; sr[1] = v.y; sr[2] = v.z; sr[3] = v.w;
    }
#if HB_RETRY_DIGEST
    // the digest the first pass stored (flags bit 0), else hash the index
    __device__ __forceinline__ bool digest(u64 job, u32 dig[8]) const {
        const HbRetry &r = A.retry[job];
        if (!(r.flags & 1u)) return false;
        const uint4 a = *reinterpret_cast<const uint4 *>(r.dig), b = *reinterpret_cast<const uint4 *>(r.dig + 4);
        dig[0] = a.x; dig[1] = a.y; dig[2] = a.z; dig[3] = a.w;
        dig[4] = b.x; dig[5] = b.y; dig[6] = b.z; dig[7] = b.w;
        return true;
    }
#endif
    __device__ __forceinline__ void accept(u64 job, const u32 F[NL]) const {
        const u64 blk = A.retry[job].blk;
        if constexpr (ALIGN == 0) {   // split wide-prime encode: F for hb_wmac_kernel
            hb_store_limbs<NL>(A.fout + blk * NL, F);
            return;
        } else {
        u32 tag[NL];
        if (NL == 8 && A.mfma) {
            // the first pass left sum_j alpha_j m_j mod p: tag = (F + part) mod p
            u32 v[NL + 1];
            u64 c = 0;
            for (int t = 0; t < NL; ++t) {
                c += (u64)F[t] + A.retry[job].part[t < 8 ? t : 0];
                v[t] = (u32)c;
                c >>= 32;
            }
            v[NL] = (u32)c;
            hb_reduce_small<NL>(v, A.mod, tag);
        } else {
            hb_block_tag<NL, ALIGN>(A.data, A.len, blk, A.C, A.ss, A.S, A.alpha_mont, A.mod, F, tag);
        }
        hb_store_tag<NL, ALIGN>(A.tags + blk * (u64)A.tw, A.tw, tag);
        }
    }
};

template <int NL, int NR, int ALIGN>
__global__ __launch_bounds__((HbEncWg<NL, ALIGN>::v), HbEncodeOcc<NL>::v) void hb_encode_retry_kernel(EncodeArgs<NL> A) {
    __shared__ __attribute__((aligned(16))) u32 lds[HB_LDS_WORDS];
    // pass 1 has completed (stream order): the count is final
    const u64 cnt = *(volatile unsigned long long *)A.retry_count;
    const u64 n = cnt < A.retry_cap ? cnt : A.retry_cap;
    if (n == 0) return;
    hb_fill_lds(lds, A.t0);
    const LaneTab L = hb_lane_tab(lds);
    RetryHandler<NL, ALIGN> h{A};
    if constexpr ((NL == 8 || ALIGN == 0) && HB_RETRY_QUAD_TAIL) hb_engine_tail<NL, NR>(h, L, A.prf, n, A.queue, hb_qchunk(A.qchunk));
    else hb_engine<NL, NR>(h, L, A.prf, n, A.queue, hb_qchunk(A.qchunk));
}

// r (NL limbs, < p) += x (NL limbs, < p) mod p
template <int NL>
__device__ __forceinline__ void hb_add_mod(u32 r[NL], const u32 *x, const ModP<NL> &M) {
    u32 v[NL + 1], o[NL];
    u64 c = 0;
    for (int t = 0; t < NL; ++t) {
        c += (u64)r[t] + x[t];
        v[t] = (u32)c;
        c >>= 32;
    }
    v[NL] = (u32)c;
    hb_reduce_small<NL>(v, M, o);
    for (int t = 0; t < NL; ++t) r[t] = o[t];
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
    __device__ __forceinline__ void fail(u64) const {}
    __device__ __forceinline__ void accept(u64 job, const u32 v[NL]) const {
        u32 *o = A.out + job * NL;
        for (int t = 0; t < NL; ++t) o[t] = v[t];
    }
};

// Static placement of a prove's quad-engine waves (A.place).  The launch
// lasts as long as its longest v chain, and a wave sharing its SIMD with
// other busy waves runs its chain up to 1.5x slower (one wave: 1,468 clocks
// per CFB-8 step; four on one SIMD: up to 2,202, scripts/ubench_latency.hip),
// so instead of racing for the job queue, each wave is given 16 jobs by
// position: v waves (nb CFB-8 steps per try) one per SIMD where they fit,
// index waves (4 steps per try for up to 2^32 tags) on the remaining SIMDs,
// two or more to a SIMD if they must.  Waves 4m .. 4m+3 of a workgroup run on
// the CU's four SIMDs (HW_ID, scripts/ubench_hwid.hip): slot s = (w & 3) * G
// + g is one SIMD and layer w >> 2 a wave on it.  Segregated when the v waves
// fit one layer and the index waves the free slots' four layers; otherwise
// balanced: v positions fill slots upward, index positions downward, which
// stacks at most ceil((nv + ni) / 4G) <= 4 waves on a slot (the host places
// only when nv + ni <= 16 G).  Returns 1 (v), 2 (index) or 0 (no jobs) and
// the wave's first job.
__device__ __forceinline__ int hb_prove_place(u32 G, u32 g, u32 w, u64 n, bool idx_too, u64 &first) {
    const u64 S4 = 4ull * G, s = (u64)(w & 3u) * G + g, layer = w >> 2;
    const u64 nv = (n + 15) / 16, ni = idx_too ? nv : 0;
    const u64 F = nv < S4 ? S4 - nv : 0;
    if (nv <= S4 && (ni == 0 || ni <= 4 * F)) {
        if (s < nv) {
            if (layer != 0) return 0;
            first = 16 * s;
            return 1;
        }
        const u64 j = layer * F + (s - nv);
        if (j >= ni) return 0;
        first = 16 * j;
        return 2;
    }
    const u64 cv = nv / S4 + (s < nv % S4 ? 1u : 0u);
    if (layer < cv) {
        first = 16 * (layer * S4 + s);
        return 1;
    }
    const u64 j = (layer - cv) * S4 + (S4 - 1 - s);
    if (j >= ni) return 0;
    first = 16 * j;
    return 2;
}

// QUAD: one evaluation per four lanes (hb_engine_quad, MODE 0 only) for
// latency-bound batches.
template <int NL, int NR, int MODE, bool QUAD = false>
__global__ __launch_bounds__(HB_ENGINE_WG) void hb_prf_kernel(PrfArgs<NL> A) {
    __shared__ __attribute__((aligned(16))) u32 lds[HB_LDS_WORDS];
    hb_fill_lds(lds, A.t0);
    const LaneTab L = hb_lane_tab(lds);
    PrfHandler<NL> h{A};
    if constexpr (QUAD) {
        if (A.place) {   // waves placed by SIMD (hb_prove_place), no queue
            u64 first = 0;
            if (hb_prove_place(gridDim.x, blockIdx.x, threadIdx.x >> 6, A.n, false, first) == 1)
                hb_engine_quad<NL, NR, PrfHandler<NL>>(h, L, A.prf, A.n, A.queue, A.qchunk, first);
            return;
        }
        hb_engine_quad<NL, NR, PrfHandler<NL>>(h, L, A.prf, A.n, A.queue, A.qchunk);
    } else {
        hb_engine<NL, NR, PrfHandler<NL>, MODE>(h, L, A.prf, A.n, A.queue, A.qchunk);
    }
}

// alpha_j R mod p (PySwizzle.py:291, 302), written in Montgomery form.
template <int NL>
struct AlphaMontHandler {
    const Prf2Args<NL> &A;
    __device__ __forceinline__ u64 x_of(u64 job) const { return job; }
    __device__ __forceinline__ void init(u64, u32 sr[4]) const { hb_zero_sr(sr); }
    __device__ __forceinline__ void fail(u64) const {}
    __device__ __forceinline__ void accept(u64 job, const u32 a[NL]) const {
        u32 y[NL];
        hb_to_mont<NL>(a, A.r2, A.mod, y);
        for (int t = 0; t < NL; ++t) A.amont[job * NL + t] = y[t];
    }
};

// The small-input encode's PRFs in one launch: placed quad waves (position
// p = (w >> 2) 4G + (w & 3) G + g, one wave per SIMD first), the blocks'
// F(x0 + k) on positions [0, nf) and the sectors' alpha_j on the next ones, so
// the alpha chains run beside the F chains instead of before them.
template <int NL, int NR>
__global__ __launch_bounds__(HB_ENGINE_WG) void hb_prf_pair_kernel(Prf2Args<NL> A) {
    __shared__ __attribute__((aligned(16))) u32 lds[HB_LDS_WORDS];
    hb_fill_lds(lds, A.f.t0);
    const LaneTab L = hb_lane_tab(lds);
    const u64 G = gridDim.x, w = threadIdx.x >> 6;
    const u64 pos = (w >> 2) * 4 * G + (w & 3) * G + blockIdx.x;
    const u64 nf = (A.f.n + 15) / 16, na = (A.S + 15) / 16;
    if (pos < nf) {
        PrfHandler<NL> h{A.f};
        hb_engine_quad<NL, NR, PrfHandler<NL>>(h, L, A.f.prf, A.f.n, A.f.queue, A.f.qchunk, 16 * pos);
    } else if (pos < nf + na) {
        AlphaMontHandler<NL> h{A};
        hb_engine_quad<NL, NR, AlphaMontHandler<NL>>(h, L, A.pa, A.S, A.aqueue, A.f.qchunk, 16 * (pos - nf));
    }
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

// ------------------------------------------------------------------ prove stage 1: PRFs
// idx_i = KeyedPRF(key, #tags)(i0 + i) and v_i = KeyedPRF(key, v_max)(i0 + i)
// (PySwizzle.py:344-345, 353, 357; cxx shacham_waters_private.cxx:742-748,
// 762, 767) for i < n in ONE launch: two engine runs over the same LDS image,
// v stored in Montgomery form (v R mod p) for stage 2.  check_all (cxx prove
// with a challenge covering every block, :754-762) skips the index PRF.
// Block ix of the file -- its S sectors as full ss-byte big-endian integers
// (a short last sector right-aligned, sectors past EOF zero: the reference's
// seek/read per sector, PySwizzle.py:353-360) and its tag -- copied to slot
// job of the compact gather buffers: the device twin of the host gather
// (hb_runtime.cpp, Gather::run).  One lane; whole-block 16-byte copies when
// the block lies inside the file and everything is 16-byte aligned.
__device__ __forceinline__ void hb_gather_to(const unsigned char *data, u64 len, u64 C, u32 ss, u32 S,
                                             const unsigned char *tags, u32 tw, u64 ntags, u32 align16,
                                             unsigned char *dst, unsigned char *tdst, u64 ix) {
    if (ix >= ntags) {   // reported by the host (flags); summed as 0
        for (u64 b = 0; b < C; ++b) dst[b] = 0;
        for (u32 b = 0; b < tw; ++b) tdst[b] = 0;
        return;
    }
    const u64 base = ix * C;
    if (align16 && base + C <= len) {
        // eight 16-byte loads in flight before their stores
        const uint4 *s = reinterpret_cast<const uint4 *>(data + base);
        uint4 *d = reinterpret_cast<uint4 *>(dst);
        const u64 nq = C / 16;
        u64 k = 0;
        for (; k + 8 <= nq; k += 8) {   // (named values: an array of them was kept in scratch)
            const uint4 v0 = s[k], v1 = s[k + 1], v2 = s[k + 2], v3 = s[k + 3];
            const uint4 v4 = s[k + 4], v5 = s[k + 5], v6 = s[k + 6], v7 = s[k + 7];
            d[k] = v0;
            d[k + 1] = v1;
            d[k + 2] = v2;
            d[k + 3] = v3;
            d[k + 4] = v4;
            d[k + 5] = v5;
            d[k + 6] = v6;
            d[k + 7] = v7;
        }
        for (; k < nq; ++k) d[k] = s[k];
    } else {
        for (u32 j = 0; j < S; ++j) {
            const u64 pos = base + (u64)j * ss;
            const u64 r = pos >= len ? 0 : (len - pos < ss ? len - pos : ss);
            unsigned char *ds = dst + (u64)j * ss;
            for (u64 b = 0; b < ss - r; ++b) ds[b] = 0;
            for (u64 b = 0; b < r; ++b) ds[ss - r + b] = data[pos + b];
        }
    }
    const unsigned char *ts = tags + ix * (u64)tw;
    if (align16) {   // tw % 16 == 0 and 16-byte aligned tags (hb_runtime.cpp)
        for (u32 q = 0; q < tw / 16; ++q)
            reinterpret_cast<uint4 *>(tdst)[q] = reinterpret_cast<const uint4 *>(ts)[q];
    } else {
        for (u32 b = 0; b < tw; ++b) tdst[b] = ts[b];
    }
}

__device__ __forceinline__ void hb_gather_block(const unsigned char *data, u64 len, u64 C, u32 ss, u32 S,
                                                const unsigned char *tags, u32 tw, u64 ntags, u32 align16,
                                                unsigned char *gdata, unsigned char *gtags, u64 job, u64 ix) {
    hb_gather_to(data, len, C, ss, S, tags, tw, ntags, align16, gdata + job * C, gtags + job * (u64)tw, ix);
}

template <int NL>
struct ProveIdxHandler {
    const ProveArgs<NL> &A;
    __device__ __forceinline__ u64 x_of(u64 job) const { return A.i0 + job; }
    __device__ __forceinline__ void init(u64, u32 sr[4]) const { hb_zero_sr(sr); }
    __device__ __forceinline__ void fail(u64) const {}
    __device__ __forceinline__ void accept(u64 job, const u32 v[2]) const {
        const u64 ix = (u64)v[0] | ((u64)v[1] << 32);
        A.idx[job] = ix;
        // the cxx prf returns a value >= the limit after 81 tries (prf.hxx:142),
        // on which the reference's t.sigma().at(index) throws: flagged here,
        // raised by the host; stage 2 reads such a term as 0
        if (ix >= A.ntags) atomicOr(A.flags, 1u);
        // gather the challenged block while the v chains are still running
        if (A.gdata)
            hb_gather_block(A.data, A.len, A.C, A.ss, A.S, A.tags, A.tw, A.ntags, A.galign16, A.gdata, A.gtags, job,
                            ix);
    }
};

template <int NL>
struct ProveVHandler {
    const ProveArgs<NL> &A;
    __device__ __forceinline__ u64 x_of(u64 job) const { return A.i0 + job; }
    __device__ __forceinline__ void init(u64, u32 sr[4]) const { hb_zero_sr(sr); }
    __device__ __forceinline__ void fail(u64) const {}
    __device__ __forceinline__ void accept(u64 job, const u32 v[NL]) const {
        u32 y[NL];
        hb_to_mont<NL>(v, A.r2, A.mod, y);
        u32 *o = A.vm + job * NL;
        for (int t = 0; t < NL; ++t) o[t] = y[t];
    }
};


// ------------------------------------------------------------------ fused prove
// One launch for the whole PySwizzle prove of a device-resident file when
// everything fits one workgroup's LDS (hb_runtime.cpp decides, A.fuse):
// workgroup g owns jobs [j0, j1) = [n g / G, n (g + 1) / G) (<= 48), and its
// 16 waves split as
//   waves 0-2    v waves (16 jobs each), one per SIMD (hb_prove_place's HW_ID
//                order: waves 4m .. 4m+3 sit on the CU's four SIMDs)
//   waves 3,7,11 index waves, stacked on the fourth SIMD (their chains are
//                ~1/3 of a v chain: 4 CFB-8 steps per try against 32)
//   waves 12-15  summers, one per SIMD (their work is ~1 % of a SIMD's issue)
//   the rest     exit after the table fill.
// An index wave gathers job k's block and tag from HBM into LDS slot k (the
// host gather's layout) and raises iflag[k]; a v wave stores v_k R mod p in
// LDS and raises vflag[k] (workgroup-scope release / acquire).  Summer lane
// l owns column l mod ncols and jobs k = l / ncols + r * (256 / ncols): it
// polls its jobs' flags and multiply-accumulates each term as soon as both
// halves are there, so the sums ride under the v chains instead of following
// them in a second launch (hb_wsum_kernel, ~26 us at configs[4]).  Then the
// summers' residues go into per-column u64 limb sums in LDS (ds_add_u64),
// summer wave 12 -- once every producer wave and summer wave has signalled --
// adds the workgroup's limb sums into the global ones (agent-scope atomics),
// and the last workgroup to finish (agent counter) carries, reduces and
// writes the ncols results, the status word and the completion token into
// the pinned host buffer, re-zeroing the limb sums, the counter, the PRF
// slots and the flag word -- the invariants of hb_wsum_kernel (I1-I4) hold
// for fctl / facc as for ctl.  Nobody waits on anything but producers of its
// own workgroup, which never wait: no co-residency assumption across
// workgroups.  Every job raises its flags, abandoned ones too (h.fail); the
// waits are bounded anyway (HB_FUSE_SPINS polls, ~0.4 s), and a timeout
// raises flag bit 2 -> status bit 4 -> a loud error on the host.
#ifndef HB_FUSE_SPINS
#define HB_FUSE_SPINS (1u << 22)
#endif

struct HbFz {
    u32 *iflag, *vflag, *ctr;     // ctr[0] producer waves done, [1] summer waves done, [2] timeout
    u32 *v;
    unsigned long long *acc;
    unsigned char *blk, *tag;
};

template <int NL>
__device__ __forceinline__ HbFz hb_fz(unsigned char *base, const ProveArgs<NL> &A) {
    u32 off[5];
    hb_fz_layout(A.fcmax, NL, A.ncols, A.C, A.tw, off);
    HbFz z;
    z.iflag = (u32 *)base;
    z.vflag = z.iflag + A.fcmax;
    z.ctr = z.vflag + A.fcmax;
    z.v = (u32 *)(base + off[1]);
    z.acc = (unsigned long long *)(base + off[2]);
    z.blk = base + off[3];
    z.tag = base + off[4];
    return z;
}

__device__ __forceinline__ void hb_fz_raise(u32 *flag) {
    __hip_atomic_store(flag, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ u32 hb_fz_get(const u32 *flag) {
    return __hip_atomic_load(flag, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
}

template <int NL>
struct FusedIdxHandler {
    const ProveArgs<NL> &A;
    const HbFz &z;
    u64 j0;
    __device__ __forceinline__ u64 x_of(u64 job) const { return A.i0 + job; }
    __device__ __forceinline__ void init(u64, u32 sr[4]) const { hb_zero_sr(sr); }
    __device__ __forceinline__ void gather(u64 job, u64 ix) const {
        const u64 k = job - j0;
        hb_gather_to(A.data, A.len, A.C, A.ss, A.S, A.tags, A.tw, A.ntags, A.galign16, z.blk + k * A.C,
                     z.tag + k * (u64)A.tw, ix);
        hb_fz_raise(z.iflag + k);
    }
    __device__ __forceinline__ void accept(u64 job, const u32 v[2]) const {
        const u64 ix = (u64)v[0] | ((u64)v[1] << 32);
        if (ix >= A.ntags) atomicOr(A.flags, 1u);   // as ProveIdxHandler; summed as 0
        gather(job, ix);
    }
    __device__ __forceinline__ void fail(u64 job) const { gather(job, A.ntags); }   // zeros; status bit 2
};

template <int NL, class ARGS = ProveArgs<NL>>
struct FusedVHandler {
    const ARGS &A;
    const HbFz &z;
    u64 j0;
    __device__ __forceinline__ u64 x_of(u64 job) const { return A.i0 + job; }
    __device__ __forceinline__ void init(u64, u32 sr[4]) const { hb_zero_sr(sr); }
    __device__ __forceinline__ void accept(u64 job, const u32 v[NL]) const {
        u32 y[NL];
        hb_to_mont<NL>(v, A.r2, A.mod, y);
        u32 *o = z.v + (job - j0) * NL;
        for (int t = 0; t < NL; ++t) o[t] = y[t];
        hb_fz_raise(z.vflag + (job - j0));
    }
    __device__ __forceinline__ void fail(u64 job) const {
        u32 *o = z.v + (job - j0) * NL;
        for (int t = 0; t < NL; ++t) o[t] = 0;
        hb_fz_raise(z.vflag + (job - j0));
    }
};

// The common end of a fused launch's summer waves (12 .. 15): each summer
// lane that had terms (have) reduces its sum once and adds the residue into
// the workgroup's per-column u64 limb sums in LDS; when all four summer waves
// and the workgroup's nprod producer waves have signalled, wave 12 adds the
// limb sums into the global ones and bumps the workgroup counter; the last
// workgroup carries and reduces the nc sums (< 2^16 p), writes them, the
// status word (bit 1: a PRF job abandoned in any of the nslots engine slots;
// flags bits 0 and 2) and -- after a system-scope release -- the completion
// token into `out`, and re-zeroes facc, the counter, the slots and the flags.
template <int NL>
__device__ __forceinline__ void hb_fused_close(const ModP<NL> &mod, const HbFz &z, bool have, u32 acc[2 * NL + 1],
                                               u32 col, bool timeout, u32 nc, u32 nprod,
                                               unsigned long long *facc, unsigned int *fctl, u32 *out, u32 token,
                                               unsigned long long *qslots, u32 nslots, unsigned int *flags) {
    if (have) {
        u32 v[NL + 1], res[NL];
        hb_redc<NL>(acc, mod, v);
        hb_reduce_small<NL>(v, mod, res);
        for (int t = 0; t < NL; ++t)
            __hip_atomic_fetch_add(z.acc + col * NL + t, (unsigned long long)res[t], __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_WORKGROUP);
    }
    if (__ballot(timeout)) {
        if (hb_lane_id() == 0) __hip_atomic_store(z.ctr + 2, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    if (hb_lane_id() == 0) __hip_atomic_fetch_add(z.ctr + 1, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
    if (threadIdx.x >> 6 != 12) return;
    // wave 12: every summer and producer wave of this workgroup has signalled
    u32 spins = 0;
    while (__hip_atomic_load(z.ctr + 1, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) < 4u ||
           __hip_atomic_load(z.ctr + 0, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) < nprod) {
        if (++spins > HB_FUSE_SPINS) {
            timeout = true;
            break;
        }
        __builtin_amdgcn_s_sleep(2);
    }
    for (u32 i = hb_lane_id(); i < nc * NL; i += 64) {
        const unsigned long long x = __hip_atomic_load(z.acc + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        if (x) __hip_atomic_fetch_add(facc + i, x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    const bool to = __ballot(timeout) != 0 || __hip_atomic_load(z.ctr + 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    if (to && hb_lane_id() == 0) atomicOr(flags, 4u);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    u32 lastw = 0;
    if (hb_lane_id() == 0)
        lastw = __hip_atomic_fetch_add(fctl, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT) + 1u == gridDim.x;
    if (!__builtin_amdgcn_readfirstlane(lastw)) return;
    // the last workgroup: carry, reduce and write the nc sums, re-zero
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    for (u32 c = hb_lane_id(); c < nc; c += 64) {
        u32 v[NL + 1], o[NL];
        u64 carry = 0;
        for (int t = 0; t < NL; ++t) {
            unsigned long long *a = facc + c * NL + t;
            carry += __hip_atomic_load(a, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(a, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            v[t] = (u32)carry;
            carry >>= 32;
        }
        v[NL] = (u32)carry;      // < 2^16 p in all: <= 256 residues < p per workgroup
        hb_reduce_small<NL>(v, mod, o);
        for (int t = 0; t < NL; ++t) out[(u64)c * NL + t] = o[t];
    }
    if (hb_lane_id() == 0) {
        u32 st = 0;
        for (u32 q = 0; q < nslots; ++q) {
            unsigned long long *qs = qslots + (u64)q * HB_QSLOT;
            st |= __hip_atomic_load(qs + 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ? 2u : 0u;
            for (int k2 = 0; k2 < HB_QSLOT; ++k2) __hip_atomic_store(qs + k2, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        const u32 fl = __hip_atomic_load(flags, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        st |= (fl & 1u) | ((fl & 4u) ? 4u : 0u);
        __hip_atomic_store(flags, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(fctl, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        out[(u64)nc * NL] = st;
    }
    // the token last, after a system-scope release: the host may poll it in
    // the pinned buffer and read the sums as soon as it changes (finish_sums)
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
    if (hb_lane_id() == 0)
        __hip_atomic_store(out + (u64)nc * NL + 1, token, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// Summer wave (12 .. 15) of the fused prove.
template <int NL>
__device__ __forceinline__ void hb_fused_sum(const ProveArgs<NL> &A, const HbFz &z, u64 j0, u64 j1) {
    const u32 l = threadIdx.x - 12u * 64u, nc = A.ncols, R = 256u / nc;
    const u32 col = l % nc, r = l / nc, cnt = (u32)(j1 - j0);
    bool timeout = false;
    u32 acc[2 * NL + 1];
    for (int t = 0; t <= 2 * NL; ++t) acc[t] = 0;
    if (r < R) {
        u64 pending = 0;
        for (u32 k = r; k < cnt; k += R) pending |= 1ull << k;
        u32 spins = 0;
        while (pending) {
            u64 pm = pending;
            bool any = false;
            while (pm) {
                const u32 k = (u32)__builtin_ctzll(pm);
                pm &= pm - 1;
                if (!hb_fz_get(z.vflag + k) || !hb_fz_get(z.iflag + k)) continue;
                u32 m[NL];
                if (col < A.S) {
                    const u64 off = (u64)k * A.C + (u64)col * A.ss;
                    if (A.fsec16) hb_load_full16<NL>(z.blk, off, m);
                    else hb_load_be_bytes<NL>(z.blk, off, A.ss, m);
                } else {
                    if (A.ftag16) hb_load_full16<NL>(z.tag, (u64)k * A.tw, m);
                    else hb_load_be_bytes<NL>(z.tag, (u64)k * A.tw, A.tw, m);
                }
                hb_mac<NL>(acc, z.v + (u64)k * NL, m);
                pending &= ~(1ull << k);
                any = true;
            }
            if (!any) {
                if (++spins > HB_FUSE_SPINS) {
                    timeout = true;
                    break;
                }
                __builtin_amdgcn_s_sleep(2);
            }
        }
    }
    hb_fused_close<NL>(A.mod, z, r < R, acc, col, timeout, nc, 6u, A.facc, A.fctl, A.fout, A.ftoken, A.queue, 2u,
                       A.flags);
}

template <int NL, int NR>
__device__ __forceinline__ void hb_prove_fused(const ProveArgs<NL> &A, const LaneTab &L, const HbFz &z) {
    const u64 G = gridDim.x, g = blockIdx.x;
    const u64 j0 = A.n * g / G, j1 = A.n * (g + 1) / G;
    const u32 w = threadIdx.x >> 6;
    if (w < 4 || w == 7 || w == 11) {
        const bool isv = w < 3;
        const u64 first = j0 + 16ull * (isv ? w : w >> 2);
        if (first < j1) {
            if (isv) {
                FusedVHandler<NL> h{A, z, j0};
                hb_engine_quad<NL, NR, FusedVHandler<NL>>(h, L, A.pv, A.n, A.queue + HB_QSLOT, A.qchunk, first, j1);
            } else {
                FusedIdxHandler<NL> h{A, z, j0};
                hb_engine_quad<2, NR, FusedIdxHandler<NL>>(h, L, A.pi, A.n, A.queue, A.qchunk, first, j1);
            }
        }
        // the engine's statistics (q[1], q[2]) before the signal
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        if (hb_lane_id() == 0) __hip_atomic_fetch_add(z.ctr, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
    } else if (w >= 12) {
        hb_fused_sum<NL>(A, z, j0, j1);
    }
}

// ------------------------------------------------------------------ fused verify
// PySwizzle.verify's right-hand side (PySwizzle.py:380-395) in one launch,
// on the fused prove's scheme (hb_prove_fused): workgroup g owns challenge
// jobs [n g / G, n (g + 1) / G) (<= 48);
//   waves 0-2  v = KeyedPRF(chal_key, v_max)(i), v R mod p into LDS (+ flag)
//   waves 3-5  idx = KeyedPRF(chal_key, #chunks)(i) for their 16 jobs, then
//              F = KeyedPRF(f_key, p)(idx) (a quad engine over the same jobs
//              whose inputs are those indices) into LDS (+ flag): serial in
//              the wave, the index chains being ~1/4 of an F chain
//   wave 6     alpha_j = KeyedPRF(alpha_key, p)(j), j in [16 g, 16 g + 16) of
//              [0, S), and the terms alpha_j mu_j straight into the
//              workgroup's limb sums
//   waves 12-15 summers: lane k adds v_k F_k as soon as both are there.
// 7 producer waves signal; the close is hb_fused_close's (one column).
// Long chains: 3 v + 3 F waves per CU on its 4 SIMDs (waves 3..5 sit on
// SIMDs 3, 0, 1), so two SIMDs host two.
template <int NL>
__device__ __forceinline__ HbFz hb_fz_verify(unsigned char *base, const VerifyArgs<NL> &A) {
    u32 off[5];
    hb_fz_layout(A.fcmax, NL, 1, 4ull * NL, 8, off);   // "blocks": F slots, "tags": index slots
    HbFz z;
    z.iflag = (u32 *)base;       // F ready
    z.vflag = z.iflag + A.fcmax;
    z.ctr = z.vflag + A.fcmax;
    z.v = (u32 *)(base + off[1]);
    z.acc = (unsigned long long *)(base + off[2]);
    z.blk = base + off[3];
    z.tag = base + off[4];
    return z;
}

template <int NL>
struct VerifyIdxHandler {
    const VerifyArgs<NL> &A;
    const HbFz &z;
    u64 j0;
    __device__ __forceinline__ u64 x_of(u64 job) const { return A.i0 + job; }
    __device__ __forceinline__ void init(u64, u32 sr[4]) const { hb_zero_sr(sr); }
    __device__ __forceinline__ void accept(u64 job, const u32 v[2]) const {
        reinterpret_cast<u64 *>(z.tag)[job - j0] = (u64)v[0] | ((u64)v[1] << 32);
    }
    __device__ __forceinline__ void fail(u64 job) const { reinterpret_cast<u64 *>(z.tag)[job - j0] = 0; }
};

template <int NL>
struct VerifyFHandler {   // F(idx) (PySwizzle.py:389): the input is the job's index
    const VerifyArgs<NL> &A;
    const HbFz &z;
    u64 j0;
    __device__ __forceinline__ u64 x_of(u64 job) const { return reinterpret_cast<const u64 *>(z.tag)[job - j0]; }
    __device__ __forceinline__ void init(u64, u32 sr[4]) const { hb_zero_sr(sr); }
    __device__ __forceinline__ void accept(u64 job, const u32 f[NL]) const {
        u32 *o = reinterpret_cast<u32 *>(z.blk) + (job - j0) * NL;
        for (int t = 0; t < NL; ++t) o[t] = f[t];
        hb_fz_raise(z.iflag + (job - j0));
    }
    __device__ __forceinline__ void fail(u64 job) const {
        u32 *o = reinterpret_cast<u32 *>(z.blk) + (job - j0) * NL;
        for (int t = 0; t < NL; ++t) o[t] = 0;
        hb_fz_raise(z.iflag + (job - j0));
    }
};

template <int NL>
struct VerifyAlphaHandler {   // alpha_j mu_j (PySwizzle.py:392) into the limb sums
    const VerifyArgs<NL> &A;
    const HbFz &z;
    __device__ __forceinline__ u64 x_of(u64 job) const { return job; }
    __device__ __forceinline__ void init(u64, u32 sr[4]) const { hb_zero_sr(sr); }
    __device__ __forceinline__ void accept(u64 job, const u32 a[NL]) const {
        u32 y[NL], m[NL], acc[2 * NL + 1], v[NL + 1], res[NL];
        hb_to_mont<NL>(a, A.r2, A.mod, y);
        for (int t = 0; t < NL; ++t) m[t] = A.mu[job * NL + t];
        for (int t = 0; t <= 2 * NL; ++t) acc[t] = 0;
        hb_mac<NL>(acc, y, m);
        hb_redc<NL>(acc, A.mod, v);
        hb_reduce_small<NL>(v, A.mod, res);
        for (int t = 0; t < NL; ++t)
            __hip_atomic_fetch_add(z.acc + t, (unsigned long long)res[t], __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_WORKGROUP);
    }
    __device__ __forceinline__ void fail(u64) const {}   // status bit 1 (abandoned job)
};

template <int NL, int NR>
__global__ __launch_bounds__(HB_ENGINE_WG) void hb_verify_fused_kernel(VerifyArgs<NL> A) {
    __shared__ __attribute__((aligned(16))) u32 lds[HB_LDS_WORDS];
    __shared__ __attribute__((aligned(16))) unsigned char fz[HB_FZ_BYTES];
    const HbFz z = hb_fz_verify<NL>(fz, A);
    for (u32 i = threadIdx.x; i < 2 * A.fcmax + 4; i += blockDim.x) z.iflag[i] = 0;
    for (u32 i = threadIdx.x; i < NL; i += blockDim.x) z.acc[i] = 0;
    hb_fill_lds(lds, A.t0);
    const LaneTab L = hb_lane_tab(lds);
    const u64 G = gridDim.x, g = blockIdx.x;
    const u64 j0 = A.n * g / G, j1 = A.n * (g + 1) / G;
    const u32 w = threadIdx.x >> 6;
    if (w < 7) {
        if (w < 3) {
            const u64 first = j0 + 16ull * w;
            if (first < j1) {
                FusedVHandler<NL, VerifyArgs<NL>> h{A, z, j0};
                hb_engine_quad<NL, NR, FusedVHandler<NL, VerifyArgs<NL>>>(h, L, A.pv, A.n, A.queue + HB_QSLOT,
                                                                          A.qchunk, first, j1);
            }
        } else if (w < 6) {
            const u64 first = j0 + 16ull * (w - 3);
            if (first < j1) {
                VerifyIdxHandler<NL> hi{A, z, j0};
                hb_engine_quad<2, NR, VerifyIdxHandler<NL>>(hi, L, A.pi, A.n, A.queue, A.qchunk, first, j1);
                VerifyFHandler<NL> hf{A, z, j0};
                hb_engine_quad<NL, NR, VerifyFHandler<NL>>(hf, L, A.pf, A.n, A.queue + 2 * HB_QSLOT, A.qchunk, first,
                                                           j1);
            }
        } else {
            const u64 first = 16ull * g;
            if (first < A.S) {
                VerifyAlphaHandler<NL> ha{A, z};
                hb_engine_quad<NL, NR, VerifyAlphaHandler<NL>>(ha, L, A.pa, A.S, A.queue + 3 * HB_QSLOT, A.qchunk,
                                                               first, A.S);
            }
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        if (hb_lane_id() == 0) __hip_atomic_fetch_add(z.ctr, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
    } else if (w >= 12) {
        const u32 k = threadIdx.x - 12u * 64u, cnt = (u32)(j1 - j0);
        bool timeout = false;
        u32 acc[2 * NL + 1];
        for (int t = 0; t <= 2 * NL; ++t) acc[t] = 0;
        if (k < cnt) {
            u32 spins = 0;
            while (!hb_fz_get(z.vflag + k) || !hb_fz_get(z.iflag + k)) {
                if (++spins > HB_FUSE_SPINS) {
                    timeout = true;
                    break;
                }
                __builtin_amdgcn_s_sleep(2);
            }
            if (!timeout) hb_mac<NL>(acc, z.v + (u64)k * NL, reinterpret_cast<const u32 *>(z.blk) + (u64)k * NL);
        }
        hb_fused_close<NL>(A.mod, z, k < cnt, acc, 0u, timeout, 1u, 7u, A.facc, A.fctl, A.fout, A.ftoken, A.queue,
                           4u, A.flags);
    }
}

template <int NL, int NR, int MODE_I, int MODE_V, bool QUAD = false>
__global__ __launch_bounds__(HB_ENGINE_WG) void hb_prove_prf_kernel(ProveArgs<NL> A) {
    __shared__ __attribute__((aligned(16))) u32 lds[HB_LDS_WORDS];
    if constexpr (QUAD) {
        if (A.fuse) {
            __shared__ __attribute__((aligned(16))) unsigned char fz[HB_FZ_BYTES];
            const HbFz z = hb_fz<NL>(fz, A);
            // flags, counters and limb sums start at zero (ordered by the fill's barrier)
            for (u32 i = threadIdx.x; i < 2 * A.fcmax + 4; i += blockDim.x) z.iflag[i] = 0;
            for (u32 i = threadIdx.x; i < A.ncols * NL; i += blockDim.x) z.acc[i] = 0;
            hb_fill_lds(lds, A.t0);
            hb_prove_fused<NL, NR>(A, hb_lane_tab(lds), z);
            return;
        }
    }
    hb_fill_lds(lds, A.t0);
    const LaneTab L = hb_lane_tab(lds);
    if constexpr (QUAD) {
        if (A.place) {
            u64 first = 0;
            const int role = hb_prove_place(gridDim.x, blockIdx.x, threadIdx.x >> 6, A.n, !A.check_all, first);
            if (role == 1) {
                ProveVHandler<NL> hv{A};
                hb_engine_quad<NL, NR, ProveVHandler<NL>>(hv, L, A.pv, A.n, A.queue + HB_QSLOT, A.qchunk, first);
            } else if (role == 2) {
                ProveIdxHandler<NL> hi{A};
                hb_engine_quad<2, NR, ProveIdxHandler<NL>>(hi, L, A.pi, A.n, A.queue, A.qchunk, first);
            }
            return;
        }
    }
    // The two PRFs run side by side on disjoint halves of the grid: the
    // launch lasts as long as its longest rejection chain (a serial CFB
    // stream), and running the index chain before the v chain in the same
    // waves would add the two.
    const bool idx_half = !A.check_all && gridDim.x > 1 && blockIdx.x < gridDim.x / 2;
    if (!A.check_all && (idx_half || gridDim.x == 1)) {
        ProveIdxHandler<NL> hi{A};
        if constexpr (QUAD) hb_engine_quad<2, NR, ProveIdxHandler<NL>>(hi, L, A.pi, A.n, A.queue, A.qchunk);
        else hb_engine<2, NR, ProveIdxHandler<NL>, MODE_I>(hi, L, A.pi, A.n, A.queue, A.qchunk);
    }
    if (!idx_half) {
        ProveVHandler<NL> hv{A};
        if constexpr (QUAD) hb_engine_quad<NL, NR, ProveVHandler<NL>>(hv, L, A.pv, A.n, A.queue + HB_QSLOT, A.qchunk);
        else hb_engine<NL, NR, ProveVHandler<NL>, MODE_V>(hv, L, A.pv, A.n, A.queue + HB_QSLOT, A.qchunk);
    }
}

// ------------------------------------------------------------------ prove stage 2 / verify: weighted sums
// Sector value at absolute offset pos: BE(data[pos : min(pos + ss, len)]),
// 0 past EOF -- a short (last) sector is right-aligned, and the reference's
// break after a short read (PySwizzle.py:359-360) only skips sectors past EOF.
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

// sh[k*(NL+1) ..]: n values of NL+1 limbs (whose total fits NL+1 limbs);
// leaves their sum in sh[0 .. NL].  Block-wide call.
template <int NL>
__device__ __forceinline__ void hb_tree_sum(u32 *sh, u32 n) {
    for (u32 sft = n / 2; sft > 0; sft >>= 1) {
        if (threadIdx.x < sft) {
            u32 *x = sh + threadIdx.x * (NL + 1);
            const u32 *y = sh + (threadIdx.x + sft) * (NL + 1);
            u64 c = 0;
            for (int t = 0; t <= NL; ++t) {
                c += (u64)x[t] + y[t];
                x[t] = (u32)c;
                c >>= 32;
            }
        }
        __syncthreads();
    }
}

// column col of the weighted sum, term i:  w_i * value_col(i)
//   mode 0 (prove, device-resident file): col < S -> sector col of block idx_i
//          (absolute offset idx_i*C + col*ss, unsigned int arithmetic in the
//          cxx prove, :762-763), col == S -> tag idx_i
//   mode 1 (verify): single column, value = vals[i]
//   mode 2 (prove, host-gathered batch): sector col of gathered block i (full
//          ss-byte big-endian integers), col == S -> gathered tag i
// Each thread accumulates its terms exactly (2NL+1 limbs) and reduces once;
// a workgroup tree-reduces its residues; the last workgroup of each column
// (agent-scope counter) adds the column's partials into out[col] (or onto it,
// `accumulate`, for host batches after the first).  The call with `finalize`
// also records the PRF engines' abandoned-job counts and the index flags in
// out[ncols*NL] and zeroes the counters for the next operation: a prove is
// two launches with no memset.
//
// Cross-workgroup protocol and the invariants it rests on (a result is only
// as good as these):
//  I1  ctl[0 .. ncols] are 0 when a launch starts.  Established by the
//      allocation memset (hb_runtime.cpp ensure_ctl) and re-established by
//      every launch that runs to its end: each column's finisher stores
//      ctl[col] = 0 after the column's last increment, the closer (the last
//      column to finish) stores ctl[ncols] = 0; a prove cut short between
//      its launches makes the host clear them (prove_dirty).  Every
//      workgroup increments its column's counter exactly once (no path
//      returns before the increment), so in a launch that starts with I1 the
//      counter of every column reaches gridDim.x exactly once.
//  I2  Partials are published before the counter (release) and read by the
//      finisher after it (acquire), both at agent scope.
//  I3  out[] is written only by column finishers and the closer, and read by
//      the host (or an `accumulate` launch) only after the launch completed
//      (stream order).
//  I4  The PRF slots and the index flag word are read and cleared once per
//      operation, by the closer of the finalizing launch, after every column
//      is done (the PRF kernel that wrote them precedes in stream order).
// If I1 fails, a column's finisher does not run (a stale count >= gridDim.x
// means the column's counter never hits gridDim.x) or runs early, and out[col]
// silently keeps what it held before -- the round-4 failure of an
// experimental variant (profiles/r04/q/gpu_tests_wsa_early_status_only.log):
// the first 2048-bit prove of the process, one workgroup per column, returned
// a mu of an empty file that was not a sum at all but stale memory (words 0,
// 16 and 24 = 0x7f / 0x9f / 0x7f, the layout of the engine-queue counters;
// the same words in two runs with different histories): out[0 .. NL) as the
// host read it was not written by that launch's column finisher -- either the
// finisher did not run (I1 broken) or its result never reached the host's
// freshly grown read-back buffer; the data cannot tell which.  (The variant's
// source was not kept, so the write that broke it is not named here; the
// shipped kernel keeps I1 by the resets above.)
// So the host no longer trusts a result the closer did not vouch for: every
// launch's closer writes out[ncols*NL + 1] = token (distinct per launch,
// never 0) -- an `accumulate` launch only if the word still holds the
// previous launch's token (token - 1), else 0 -- and the host rejects the
// result unless the word equals the last launch's token (finish_sums; the
// token travels in the same read-back as the sums).  A launch in which some
// column never finished, a batch chain with a gap, or a read-back that did
// not land is thereby a loud error, not a wrong proof.
template <int NL, int ALIGN>
__global__ __launch_bounds__(HB_WSUM_WG) void hb_wsum_kernel(WsumArgs<NL> A) {
    __shared__ u32 sh[HB_WSUM_WG * (NL + 1)];
    __shared__ unsigned int last;
    const u32 col = blockIdx.y;
    const u64 tid = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    const u64 nthreads = (u64)gridDim.x * blockDim.x;
    u32 acc[2 * NL + 1];
    for (int t = 0; t <= 2 * NL; ++t) acc[t] = 0;
    u32 m[NL];
    for (u64 i = tid; i < A.nterms; i += nthreads) {
        if (A.mode == 1) {
            for (int t = 0; t < NL; ++t) m[t] = A.vals[i * NL + t];
        } else if (A.mode == 2) {
            if (col < A.S) hb_load_full16_or_bytes<NL, ALIGN>(A.data, i * A.C + (u64)col * A.ss, A.ss, m);
            else hb_load_be_bytes<NL>(A.tags, i * A.tw, A.tw, m);
        } else {
            const u64 blk = A.idx ? A.idx[i] : A.idx_base + i;
            if (blk >= A.ntags) {
                for (int t = 0; t < NL; ++t) m[t] = 0;
            } else if (col < A.S) {
                const u64 pos = A.wrap32 ? (u64)(u32)(blk * A.C + (u64)col * A.ss) : blk * A.C + (u64)col * A.ss;
                hb_sector_value<NL, ALIGN>(A.data, A.len, pos, A.ss, m);
            } else {
                hb_load_be_bytes<NL>(A.tags, blk * A.tw, A.tw, m);
            }
        }
        hb_mac<NL>(acc, A.w + i * NL, m);
    }
    u32 v[NL + 1], r[NL];
    hb_redc<NL>(acc, A.mod, v);
    hb_reduce_small<NL>(v, A.mod, r);
    // workgroup tree sum of the residues: plain (NL+1)-limb adds, < 256 p,
    // one reduction at the end
    for (int t = 0; t < NL; ++t) sh[threadIdx.x * (NL + 1) + t] = r[t];
    sh[threadIdx.x * (NL + 1) + NL] = 0;
    __syncthreads();
    hb_tree_sum<NL>(sh, blockDim.x);
    u32 *part = A.partials + ((u64)col * gridDim.x + blockIdx.x) * NL;
    if (threadIdx.x == 0) {
        for (int t = 0; t <= NL; ++t) v[t] = sh[t];
        hb_reduce_small<NL>(v, A.mod, r);
        for (int t = 0; t < NL; ++t) part[t] = r[t];
    }
    __syncthreads();
    // the last workgroup of this column finishes it (release / acquire at agent scope)
    if (threadIdx.x == 0) {
        const unsigned int k = __hip_atomic_fetch_add(A.ctl + col, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
        last = k + 1 == gridDim.x;
    }
    __syncthreads();
    if (!last) return;
    // the column's gridDim.x (<= blockDim.x) partials, summed in parallel
    for (int t = 0; t <= NL; ++t) sh[threadIdx.x * (NL + 1) + t] = 0;
    if (threadIdx.x < gridDim.x) {
        const u32 *pp = A.partials + ((u64)col * gridDim.x + threadIdx.x) * NL;
        for (int t = 0; t < NL; ++t)
            sh[threadIdx.x * (NL + 1) + t] = __hip_atomic_load(pp + t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __syncthreads();
    hb_tree_sum<NL>(sh, blockDim.x);
    if (threadIdx.x == 0) {
        u32 sum[NL];
        for (int t = 0; t <= NL; ++t) v[t] = sh[t];
        hb_reduce_small<NL>(v, A.mod, sum);
        if (A.accumulate) hb_add_mod<NL>(sum, A.out + (u64)col * NL, A.mod);
        for (int t = 0; t < NL; ++t) A.out[(u64)col * NL + t] = sum[t];
        A.ctl[col] = 0;
        // the last column to finish closes the operation
        const unsigned int d = __hip_atomic_fetch_add(A.ctl + A.ncols, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
        if (d + 1 == A.ncols) {
            A.ctl[A.ncols] = 0;
            // completion token (see above): every column of this launch is done
            u32 *tok = A.out + (u64)A.ncols * NL + 1;
            *tok = !A.accumulate || *tok == A.token - 1u ? A.token : 0u;
            if (A.finalize) {
                u32 st = 0;
                for (u32 s = 0; s < A.nslots; ++s) {
                    unsigned long long *q = A.qslots + (u64)s * HB_QSLOT;
                    st |= q[2] ? 2u : 0u;
                    for (int k2 = 0; k2 < HB_QSLOT; ++k2) q[k2] = 0;
                }
                if (A.flags) {
                    st |= *A.flags;
                    *A.flags = 0;
                }
                A.out[(u64)A.ncols * NL] = st;
            }
            __threadfence();
        }
    }
}

// ------------------------------------------------------------------ launchers
// Plain C++ entry points for hb_runtime.cpp (explicit instantiation per
// limb count NL, AES rounds NR and sector alignment class).  While the
// calling thread has hb_load_only set (hb_ctx_prepare, HbLoadOnly in
// hb_runtime.cpp) a launcher launches nothing: it only makes the runtime load
// the kernel's code object, which otherwise happens inside the first launch.
// Otherwise a grid with a zero dimension is an error, never a silent no-op.
template <class K>
__host__ inline void hb_load_kernel(K *k) {
    hipFuncAttributes fa;
    (void)hipFuncGetAttributes(&fa, reinterpret_cast<const void *>(k));
}
#define HB_LAUNCH(KT, G, B, S, A)                                          \
    do {                                                                   \
        if (hb_load_only) hb_load_kernel(&KT);                             \
        else if (!(G).x || !(G).y) return hipErrorInvalidConfiguration;    \
        else hipLaunchKernelGGL(KT, G, B, 0, S, A);                        \
    } while (0)
// pass: 0 = single-pass engine, 1 = first tries (prefix image), 2 = retry list,
// 3 = cxx prf encode
template <int NL, int PASS>
hipError_t hb_launch_encode_pass(const EncodeArgs<NL> &A, int nr, int align, int grid, hipStream_t s) {
    dim3 g(grid);
#define HB_ENC(K, NRV, AL) HB_LAUNCH((K<NL, NRV, AL>), g, dim3(HbEncWg<NL, AL>::v), s, A)
#define HB_ENC_NR(K, AL) \
    do { if (nr == 14) HB_ENC(K, 14, AL); else if (nr == 12) HB_ENC(K, 12, AL); else HB_ENC(K, 10, AL); } while (0)
#define HB_ENC_AL(K) do { if (align == 16) HB_ENC_NR(K, 16); else HB_ENC_NR(K, 1); } while (0)
    // align 0: the split wide-prime encode's F-only passes (NL >= 16)
#define HB_ENC_AL0(K)                                              \
    do {                                                           \
        if constexpr (NL >= 16) {                                  \
            if (align == 0) { HB_ENC_NR(K, 0); break; }            \
        }                                                          \
        if (align == 0) return hipErrorInvalidValue;               \
        HB_ENC_AL(K);                                              \
    } while (0)
    if constexpr (PASS == 1) HB_ENC_AL0(hb_encode_first_kernel);
    else if constexpr (PASS == 2) HB_ENC_AL0(hb_encode_retry_kernel);
    else if constexpr (PASS == 3) HB_ENC_AL0(hb_cxx_encode_kernel);
    else HB_ENC_AL(hb_encode_kernel);
#undef HB_ENC_AL0
#undef HB_ENC_AL
#undef HB_ENC_NR
#undef HB_ENC
    return hipGetLastError();
}

template <int NL>
hipError_t hb_launch_prf_pair(const Prf2Args<NL> &A, int nr, int grid, hipStream_t s) {
    dim3 g(grid), b(HB_ENGINE_WG);
    if (nr == 14) HB_LAUNCH((hb_prf_pair_kernel<NL, 14>), g, b, s, A);
    else if (nr == 12) HB_LAUNCH((hb_prf_pair_kernel<NL, 12>), g, b, s, A);
    else HB_LAUNCH((hb_prf_pair_kernel<NL, 10>), g, b, s, A);
    return hipGetLastError();
}

template <int NL>
hipError_t hb_launch_mac(const EncodeArgs<NL> &A, int align, hipStream_t s) {
    constexpr u32 T = HbMacSplit<NL>::T;
    if (A.S >= 2 && A.S <= T && !hb_load_only) {
        const u32 bpw = T / A.S;
        const u64 g = (A.nblocks + bpw - 1) / bpw;
        if (align == 16) HB_LAUNCH((hb_mac_split_kernel<NL, 16>), dim3((u32)g), dim3(bpw * A.S), s, A);
        else HB_LAUNCH((hb_mac_split_kernel<NL, 1>), dim3((u32)g), dim3(bpw * A.S), s, A);
        return hipGetLastError();
    }
    if (hb_load_only) {
        hb_load_kernel(&hb_mac_split_kernel<NL, 16>);
        hb_load_kernel(&hb_mac_split_kernel<NL, 1>);
    }
    const u64 grid = (A.nblocks + 255) / 256;
    if (align == 16) HB_LAUNCH((hb_mac_kernel<NL, 16>), dim3((u32)grid), dim3(256), s, A);
    else HB_LAUNCH((hb_mac_kernel<NL, 1>), dim3((u32)grid), dim3(256), s, A);
    return hipGetLastError();
}

// One launcher per pass (hb_launch_encode_pass), so that the wide-limb
// kernels of each pass can be instantiated in a translation unit of their own
// (HB_INST_ENC_PASS) and built in parallel.
template <int NL>
hipError_t hb_launch_encode(const EncodeArgs<NL> &A, int nr, int align, int pass, int grid, hipStream_t s) {
    if (pass == 1) return hb_launch_encode_pass<NL, 1>(A, nr, align, grid, s);
    if (pass == 2) return hb_launch_encode_pass<NL, 2>(A, nr, align, grid, s);
    if (pass == 3) return hb_launch_encode_pass<NL, 3>(A, nr, align, grid, s);
    return hb_launch_encode_pass<NL, 0>(A, nr, align, grid, s);
}

// mode 0: KeyedPRF, 1: cxx prf (ByteCount(limit) % 16 == 0), 2: cxx prf (any
// limit), 3: KeyedPRF on the quad engine
template <int NL>
hipError_t hb_launch_prf(const PrfArgs<NL> &A, int nr, int mode, int grid, hipStream_t s) {
    dim3 g(grid), b(HB_ENGINE_WG);
#define HB_PRF_NR(M, Q)                                                               \
    do {                                                                              \
        if (nr == 14) HB_LAUNCH((hb_prf_kernel<NL, 14, M, Q>), g, b, s, A);          \
        else if (nr == 12) HB_LAUNCH((hb_prf_kernel<NL, 12, M, Q>), g, b, s, A);     \
        else HB_LAUNCH((hb_prf_kernel<NL, 10, M, Q>), g, b, s, A);                   \
    } while (0)
    if (mode == 1) {
        if constexpr (NL >= 4) HB_PRF_NR(1, false);   // cxx limits are >= 16 bytes
        else return hipErrorInvalidValue;
    } else if (mode == 2) {
        HB_PRF_NR(2, false);
    } else if (mode == 3) {
        HB_PRF_NR(0, true);
    } else {
        HB_PRF_NR(0, false);
    }
#undef HB_PRF_NR
    return hipGetLastError();
}

template <int NL>
hipError_t hb_launch_mont(const MontArgs<NL> &A, hipStream_t s) {
    const u64 grid = (A.n + 255) / 256;
    HB_LAUNCH((hb_mont_kernel<NL>), dim3((u32)grid), dim3(256), s, A);
    return hipGetLastError();
}

template <int NL>
hipError_t hb_launch_wsum(const WsumArgs<NL> &A, int align, int gridx, hipStream_t s) {
    dim3 g(gridx, A.ncols), b(HB_WSUM_WG);
    if (align == 16) HB_LAUNCH((hb_wsum_kernel<NL, 16>), g, b, s, A);
    else HB_LAUNCH((hb_wsum_kernel<NL, 1>), g, b, s, A);
    return hipGetLastError();
}

// stage 1 of prove; mode_i / mode_v: PRF modes of the index and v PRFs
// (0 KeyedPRF; cxx prf: 1 whole blocks per try, 2 any limit; 3 KeyedPRF on the
// quad engine, both)
template <int NL>
hipError_t hb_launch_prove_prf(const ProveArgs<NL> &A, int nr, int mode_i, int mode_v, int grid, hipStream_t s) {
    dim3 g(grid), b(HB_ENGINE_WG);
#define HB_PP(MI, MV, Q)                                                                          \
    do {                                                                                          \
        if (nr == 14) HB_LAUNCH((hb_prove_prf_kernel<NL, 14, MI, MV, Q>), g, b, s, A);           \
        else if (nr == 12) HB_LAUNCH((hb_prove_prf_kernel<NL, 12, MI, MV, Q>), g, b, s, A);      \
        else HB_LAUNCH((hb_prove_prf_kernel<NL, 10, MI, MV, Q>), g, b, s, A);                    \
    } while (0)
    if (mode_i == 3 && mode_v == 3) HB_PP(0, 0, true);
    else if (mode_i == 0 && mode_v == 0) HB_PP(0, 0, false);
    else if (mode_v == 2) HB_PP(2, 2, false);
    else if constexpr (NL >= 4) HB_PP(2, 1, false);
    else return hipErrorInvalidValue;
#undef HB_PP
    return hipGetLastError();
}

// fused verify (NL <= HB_FUSE_MAX_NL; every key with nr AES rounds)
template <int NL>
hipError_t hb_launch_verify_fused(const VerifyArgs<NL> &A, int nr, int grid, hipStream_t s) {
    dim3 g(grid), b(HB_ENGINE_WG);
    if (nr == 14) HB_LAUNCH((hb_verify_fused_kernel<NL, 14>), g, b, s, A);
    else if (nr == 12) HB_LAUNCH((hb_verify_fused_kernel<NL, 12>), g, b, s, A);
    else HB_LAUNCH((hb_verify_fused_kernel<NL, 10>), g, b, s, A);
    return hipGetLastError();
}

// Explicit instantiations per limb count; the encode and the PRF / prove
// halves can go to separate translation units (parallel builds of the
// slow-to-compile wide-limb kernels).
#define HB_INST_ENC(NL) \
    template hipError_t hb_launch_encode<NL>(const EncodeArgs<NL> &, int, int, int, int, hipStream_t); \
    template hipError_t hb_launch_mac<NL>(const EncodeArgs<NL> &, int, hipStream_t); \
    template hipError_t hb_launch_prf_pair<NL>(const Prf2Args<NL> &, int, int, hipStream_t);
// the encode dispatcher alone, its passes instantiated elsewhere
#define HB_EXTERN_ENC_PASSES(NL)                                                                  \
    extern template hipError_t hb_launch_encode_pass<NL, 0>(const EncodeArgs<NL> &, int, int, int, hipStream_t); \
    extern template hipError_t hb_launch_encode_pass<NL, 1>(const EncodeArgs<NL> &, int, int, int, hipStream_t); \
    extern template hipError_t hb_launch_encode_pass<NL, 2>(const EncodeArgs<NL> &, int, int, int, hipStream_t); \
    extern template hipError_t hb_launch_encode_pass<NL, 3>(const EncodeArgs<NL> &, int, int, int, hipStream_t);
#define HB_INST_ENC_PASS(NL, P) \
    template hipError_t hb_launch_encode_pass<NL, P>(const EncodeArgs<NL> &, int, int, int, hipStream_t);
#define HB_INST_PRF(NL)                                                                          \
    template hipError_t hb_launch_prf<NL>(const PrfArgs<NL> &, int, int, int, hipStream_t);      \
    template hipError_t hb_launch_mont<NL>(const MontArgs<NL> &, hipStream_t);                   \
    template hipError_t hb_launch_wsum<NL>(const WsumArgs<NL> &, int, int, hipStream_t);         \
    template hipError_t hb_launch_prove_prf<NL>(const ProveArgs<NL> &, int, int, int, int, hipStream_t);
#define HB_INST_VERIFY_FUSED(NL) \
    template hipError_t hb_launch_verify_fused<NL>(const VerifyArgs<NL> &, int, int, hipStream_t);
#define HB_INST(NL) HB_INST_ENC(NL) HB_INST_PRF(NL)
