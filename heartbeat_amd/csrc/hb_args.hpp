// hb_args.hpp -- kernel argument blocks shared by hb_kernels.hip and the host
// runtime (hb_runtime.cpp).  All passed by value (kernarg segment), so the
// round keys, modulus and range are wave-uniform scalar operands.
#pragma once
#include "hb_lane.hpp"

// Set by hb_ctx_prepare on its thread: the launchers only load code objects
// (hb_kernels.hpp, HB_LAUNCH).  Defined in hb_kern_misc.hip.
extern thread_local bool hb_load_only;

// Workgroup geometry of the PRF engine kernels: 1024 threads (16 waves) and a
// 128 KiB LDS T-table image per workgroup -> 1 workgroup (16 waves) per CU.
#ifndef HB_ENGINE_WG
#define HB_ENGINE_WG 1024
#endif
#define HB_ENGINE_WG_PER_CU 1
#ifndef HB_QUEUE_CHUNK
#define HB_QUEUE_CHUNK 256
#endif
// PRF tries after which a job is abandoned and reported (see hb_engine)
#define HB_MAX_TRIES 2048u
// job-queue counters per slot: [0] next job, [1] PRF tries, [2] abandoned jobs,
// [3] (encode first pass) evals pushed to the retry list
#define HB_QSLOT 4
// queue slots: 0 encode (first pass / single pass), 1 alpha PRF, 2-3 prove,
// 4-5 verify, 6 hb_prf_eval, 7 encode retry pass
#define HB_SLOT_RETRY 7

// An eval whose first try was rejected, left for the retry pass: its block
// (relative to the launch) and the CFB-8 shift register after that try.
// With the MFMA MAC (EncodeArgs::mfma) the first pass has already computed
// the block's sum_j alpha_j m_ij mod p: `part`, so the retry pass only adds F.
// HB_RETRY_DIGEST (default 1): evals whose first try is rejected by its
// first output word (all but ~2^-32 of them) are listed before the try with
// the SHA-256 digest of their index (flags bit 0), which the retry pass then
// reads instead of recomputing it: 1,092.3 vs 1,088.4 GiB/s with
// HB_RETRY_DIGEST=0
#ifndef HB_RETRY_DIGEST
#define HB_RETRY_DIGEST 1
#endif
struct HbRetry {
    u64 blk;
    u32 flags;
    u32 pad_;
    u32 sr[4];
    u32 part[8];
#if HB_RETRY_DIGEST
    u32 dig[8];
#endif
};

// MFMA MAC (hb_mfma_block_acc): the 256-bit sector MAC as an int8 matrix
// product; sectors per block it accepts (column sums stay inside int32)
#define HB_MFMA_MAX_S 2048u
// A-operand tiles per sector: 1 (dense reduced digits: 32 output digits) or
// 2 (HB_MFMA_TOEPLITZ, the A/B variant: 64 output digits of the unreduced
// product, half of each tile zero)
// The dense MAC's finish: one quotient-estimate reduction of T + F (the
// tiles carry alpha_j; default), or with HB_MAC_MONT (A/B variant) the
// Montgomery REDC of T + F R (the tiles carry alpha_j R): 1,100.0 vs
// 1,087.3 GiB/s for the plain finish
#if defined(HB_MFMA_TOEPLITZ)
#define HB_MFMA_NT 2
#else
#define HB_MFMA_NT 1
#endif

template <int NL>
struct EncodeArgs {
    PrfParams<NL> prf;            // F = KeyedPRF(f_key, p)
    ModP<NL> mod;
    const unsigned char *data;    // block k of this launch starts at data[k*C]
    u64 len;                      // bytes of `data` (end of file)
    u64 nblocks;
    u64 block_base;               // global index of block 0 (PRF input)
    unsigned char *tags;          // nblocks * tw big-endian bytes
    const u32 *alpha_mont;        // S * NL limbs: alpha_j R mod p
    const u32 *t0;                // 256-entry T0 table (global)
    unsigned long long *queue;    // HB_QSLOT counters, see above
    u64 C;
    u32 tw, ss, S;
    u32 o0;                       // E_fkey(0^16)[0]: keystream byte 0 of every eval
    const unsigned char *pfx;     // CFB prefix image (hb_lane.hpp), two-pass encode
    HbRetry *retry;               // retry list (two-pass encode)
    unsigned long long *retry_count;
    u64 retry_cap;
    u32 rtop;                     // top 32 bits of R (= p) in the PRF's nb-byte frame
    // MFMA MAC (256-bit primes, 32-byte aligned sectors): A-operand fragments
    // ([HB_MFMA_NT][S][64 lanes][16 B]) and the constant kz (hb_runtime.cpp,
    // mfma_tables): the 32 signed base-256 digits of r_jk = alpha_j 256^(31-k)
    // mod p, one per sector byte k (dense), kz = 128 sum_jk r_jk + p 2^w; or,
    // with HB_MFMA_TOEPLITZ, the 33-digit Toeplitz band of alpha_j R mod p and
    // kz = Q sum_j (alpha_j R mod p) mod p + p 2^268 (Q = 0x8080..80: the
    // sectors enter the product as bytes - 128).  mfma: 1 sector loads,
    // 2 whole-line loads (hb_line_loads), 3 the 16x16x64 MFMA
    // (hb_mfma16_block_acc)
    u32 mfma;
    const u32 *afrag;
    u32 kz[2 * NL + 1];
    // small inputs (hb_mac_kernel): F(block_base + k), NL limbs per block,
    // from a quad-engine PRF launch
    const u32 *fv;
    // split wide-prime encode (PRF kernels with ALIGN = 0): F(block_base + k)
    // as NL little-endian limbs at fout + k NL, for hb_wmac_kernel
    u32 *fout;
    // jobs per queue refill in the first / retry passes and the single-pass
    // engine (0: HB_QUEUE_CHUNK; hb_runtime.cpp encode_qchunk)
    u64 qchunk;
};

// The split wide-prime encode's argument blocks: hb_wide_args.hpp.

// Prefix image of one PRF key (hb_prefix_kernel).
struct PrefixArgs {
    u32 rk[60];
    const u32 *t0;
    unsigned char *out;           // HB_PFX_BYTES
};

template <int NL>
struct PrfArgs {
    PrfParams<NL> prf;
    const u64 *xs;                // inputs (device) or nullptr: x = x0 + k
    const u32 *digs;              // or SHA-256 digests of the inputs (8 big-endian words each)
    u64 x0;
    u64 n;
    u32 *out;                     // n * NL little-endian limbs
    const u32 *t0;
    unsigned long long *queue;
    u64 qchunk;                   // jobs per queue refill
    u32 place;                    // quad engine: waves placed by SIMD (hb_prove_place), no queue
};

// Small-input encode (hb_prf_pair_kernel): F(x0 + k) for the blocks (f) and
// alpha_j R mod p for the sectors in ONE launch (PySwizzle.py:291, 302).
template <int NL>
struct Prf2Args {
    PrfArgs<NL> f;
    PrfParams<NL> pa;             // alpha = KeyedPRF(alpha_key, p)
    ModP<NL> mod;
    u32 r2[NL];                   // R^2 mod p
    u64 S;
    u32 *amont;                   // S x NL limbs: alpha_j R mod p
    unsigned long long *aqueue;   // alpha's engine slot
};

template <int NL>
struct MontArgs {
    ModP<NL> mod;
    u32 r2[NL];                   // R^2 mod p
    const u32 *in;                // n * NL limbs, each < R
    u32 *out;                     // n * NL limbs: in * R mod p
    u64 n;
};

// Prove stage 1 (hb_prove_prf_kernel): the challenge's PRFs for indices
// i0 .. i0+n-1.
template <int NL>
struct ProveArgs {
    PrfParams<2> pi;              // idx = KeyedPRF(key, #tags) (cxx: prf with limit #tags)
    PrfParams<NL> pv;             // v = KeyedPRF(key, v_max)
    ModP<NL> mod;
    u32 r2[NL];                   // R^2 mod p: v -> v R mod p
    u64 i0, n, ntags;
    u32 check_all;                // cxx prove, chunks >= #tags: idx_i = i, no index PRF
    u64 *idx;                     // n block indices
    u32 *vm;                      // n * NL limbs: v_i R mod p
    const u32 *t0;
    unsigned long long *queue;    // 2 slots: index engine, v engine
    unsigned int *flags;          // bit 0: an index >= #tags (cxx prf after 81 tries)
    u64 qchunk;                   // jobs per queue refill
    u32 place;                    // quad engine: waves placed by SIMD (hb_prove_place), no queue
    // Device gather (device-resident file and tags): as each index is found,
    // block idx_i's S sectors (full ss-byte integers) and tag are copied to
    // slot i of gdata / gtags, the layout of the host gather, so that the
    // weighted sum reads one compact buffer (wsum mode 2).  gdata == nullptr: off.
    const unsigned char *data;    // the file (len bytes) and the tags (ntags x tw)
    u64 len, C;
    u32 ss, S, tw;
    u32 galign16;                 // file, tags, C and tw allow 16-byte copies
    const unsigned char *tags;
    unsigned char *gdata;         // n x C
    unsigned char *gtags;         // n x tw
    // Fused weighted sums (fuse != 0, hb_prove_fused): the index waves gather
    // their blocks into the workgroup's LDS arena, summer waves of the same
    // workgroup add the terms as their index and v arrive, and the last
    // workgroup finishes the sums -- no hb_wsum_kernel launch.
    u32 fuse;
    u32 ncols;                    // S + 1
    u32 fcmax;                    // most jobs of one workgroup (<= HB_FZ_MAXJOBS)
    u32 fsec16, ftag16;           // sectors / tags load as 16-byte words (ss == 4 NL / tw == 4 NL)
    u32 ftoken;                   // completion token (never 0), as hb_wsum_kernel's
    unsigned long long *facc;     // [ncols][NL] limb sums over workgroups, zero between launches
    unsigned int *fctl;           // finished-workgroup counter, zero between launches
    u32 *fout;                    // [ncols][NL] results, the status word, the token word
};

// The fused verify (hb_verify_fused_kernel): rhs = sum_i v_i F(idx_i) + sum_j
// alpha_j mu_j mod p (PySwizzle.py:380-395) in one launch, all four PRF
// keys with the same AES round count (NR, a template parameter).
template <int NL>
struct VerifyArgs {
    PrfParams<2> pi;              // idx = KeyedPRF(chal_key, #state chunks)
    PrfParams<NL> pv;             // v = KeyedPRF(chal_key, v_max)
    PrfParams<NL> pf;             // F = KeyedPRF(f_key, p) of idx
    PrfParams<NL> pa;             // alpha = KeyedPRF(alpha_key, p)
    ModP<NL> mod;
    u32 r2[NL];                   // R^2 mod p
    u64 i0, n, ntags;             // challenge indices [i0, i0 + n)
    u32 S, fcmax, ftoken, pad_;
    const u32 *mu;                // S x NL limbs, pinned host memory
    const u32 *t0;
    unsigned long long *queue;    // 4 engine slots: idx, v, F, alpha (zero between launches)
    unsigned int *flags;
    u64 qchunk;
    unsigned long long *facc;     // [NL] limb sums over workgroups, zero between launches
    unsigned int *fctl;           // finished-workgroup counter
    u32 *fout;                    // [NL] rhs, the status word, the token word
};

// The fused prove's LDS arena (next to the 128 KiB T-table image): byte
// offsets of [0] the per-job index / v ready flags (2 cmax words) and 4
// counters, [1] the v slots (cmax x NL words), [2] the workgroup's limb sums
// (ncols x NL u64), [3] the gathered blocks (cmax x C bytes), [4] their tags
// (cmax x tw); returns the arena's size.
#define HB_FZ_BYTES 30720
#define HB_FZ_MAXJOBS 48
// Widest prime (limbs) the fused prove and verify take.  At 32 limbs their
// summer and alpha waves spill (a 2NL+1-limb accumulator under a 1,024-thread
// workgroup's 128 VGPRs: 760 B of scratch per lane), but off the PRF chains
// that bound the launch: PySwizzle's defaults (1024-bit, 820 chunks) verify
// in 0.46-0.79 vs 0.86-1.71 ms as a launch sequence, prove 2-5 % faster
// (same box, three seeded primes and key sets; profiles/r05/f32).
#ifndef HB_FUSE_MAX_NL
#define HB_FUSE_MAX_NL 32
#endif
HB_HHD u64 hb_fz_layout(u32 cmax, u32 nl, u32 ncols, u64 C, u32 tw, u32 off[5]) {
    u64 o = (2ull * cmax + 4) * 4;
    off[0] = 0;
    o = (o + 15) & ~15ull;
    off[1] = (u32)o;
    o += (u64)cmax * nl * 4;
    o = (o + 15) & ~15ull;
    off[2] = (u32)o;
    o += (u64)ncols * nl * 8;
    o = (o + 15) & ~15ull;
    off[3] = (u32)(o < 0xffffffffull ? o : 0);
    o += (u64)cmax * C;
    o = (o + 15) & ~15ull;
    off[4] = (u32)(o < 0xffffffffull ? o : 0);
    o += (u64)cmax * tw;
    return o;
}

// Weighted sums  sum_i w_i * value_{col}(i)  mod p  (w_i in Montgomery form);
// modes: see hb_wsum_kernel.
#define HB_WSUM_WG 256
template <int NL>
struct WsumArgs {
    ModP<NL> mod;
    u32 mode, ncols;
    const u64 *idx;               // mode 0: block of term i (nullptr: idx_base + i)
    u64 idx_base;
    u64 ntags;                    // mode 0: terms with idx >= ntags read as 0
    const u32 *w;
    u64 nterms;
    const unsigned char *data;
    u64 len, C;
    u32 ss, S, tw;
    u32 wrap32;                   // cxx prove: offset = (unsigned int)(idx * C + j * ss)
                                  // (shacham_waters_private.cxx:738, 762-763)
    const unsigned char *tags;
    const u32 *vals;
    u32 *partials;                // [ncols][gridDim.x][NL]
    unsigned int *ctl;            // ncols + 1 counters, zero between launches
    u32 *out;                     // [ncols][NL] results, the status word, the token word
    u32 accumulate;               // out[col] += this launch's sum
    u32 finalize;                 // record + zero the PRF slots and flags
    unsigned long long *qslots;   // nslots PRF engine slots (HB_QSLOT counters each)
    u32 nslots;
    unsigned int *flags;
    u32 token;                    // this launch's completion token (never 0), see hb_wsum_kernel
};

// Merkle chunk positions and leaves (heartbeat/Merkle/Merkle.py:481-515),
// one lane per seed; each seed is its own AES / HMAC key.
struct MerkleArgs {
    const unsigned char *seeds;   // n seeds of seed_len bytes (device)
    u32 seed_len;                 // 16, 24 or 32 (an AES key, Merkle.py:502)
    u64 n;
    // offsets pass: KeyedPRF(seed, range).eval(0), range = filesz - chunksz + 1
    u32 R[2];                     // range, 2 little-endian limbs
    u32 nb, topmask;
    u32 dig0[8];                  // SHA-256("0") (util.py:91 of eval(0))
    u64 *offsets;                 // n chunk offsets
    // HMAC pass: HMAC-SHA256(seed, data[offsets[i] - rebase[i]...]) over chunksz bytes
    const unsigned char *data;
    u64 len;                      // readable bytes at data
    const u64 *hoff;              // n message offsets into data
    u64 chunksz;
    u32 *digests;                 // n * 8 big-endian words
    unsigned int *flags;          // bit 1: a PRF did not terminate
    const u32 *t0;
};
