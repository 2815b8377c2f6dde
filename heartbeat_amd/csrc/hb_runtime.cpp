// hb_runtime.cpp -- host runtime and C ABI of libhbswizzle.so (include/hbswizzle.h).
//
// Owns per-device state (stream, the global T0 table, job-queue counters,
// scratch buffers), prepares the uniform kernel arguments (AES key schedule,
// range, Montgomery constants), stages host data through the GPU in chunks
// (H2D copies on a copy stream overlapped with encode kernels on the compute
// stream), and converts results to big-endian byte strings.  All per-block and
// per-challenge arithmetic runs in the kernels of hb_kernels.hip; there is no
// CPU compute path.
#include <hip/hip_runtime.h>
#include <math.h>
#include <chrono>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <condition_variable>
#include <exception>
#include <memory>
#include <mutex>
#include <string>
#include <atomic>
#include <thread>
#include <vector>

#include "../../include/hbswizzle.h"
#include "hb_aes_host.hpp"
#include "hb_args.hpp"
#include "hb_wide_args.hpp"
#include "hb_bignum_host.hpp"

using namespace hbhost;

// launchers (hb_kernels.hip)
template <int NL> hipError_t hb_launch_encode(const EncodeArgs<NL> &, int, int, int, int, hipStream_t);
template <int NL> hipError_t hb_launch_mac(const EncodeArgs<NL> &, int, hipStream_t);
template <int NL> hipError_t hb_launch_prf_pair(const Prf2Args<NL> &, int, int, hipStream_t);
hipError_t hb_launch_prefix(const PrefixArgs &, int, int, hipStream_t);
template <int NL> hipError_t hb_launch_prf(const PrfArgs<NL> &, int, int, int, hipStream_t);
template <int NL> hipError_t hb_launch_mont(const MontArgs<NL> &, hipStream_t);
template <int NL> hipError_t hb_launch_wsum(const WsumArgs<NL> &, int, int, hipStream_t);
template <int NL> hipError_t hb_launch_prove_prf(const ProveArgs<NL> &, int, int, int, int, hipStream_t);
template <int NL> hipError_t hb_launch_verify_fused(const VerifyArgs<NL> &, int, int, hipStream_t);
hipError_t hb_launch_fill(unsigned char *, u64, u64, hipStream_t);
hipError_t hb_launch_read(const void *, u64, u32 *, int, hipStream_t);
hipError_t hb_launch_merkle_offsets(const MerkleArgs &, int, hipStream_t);
hipError_t hb_launch_hmac(const MerkleArgs &, hipStream_t);
template <int NL> hipError_t hb_launch_wtab(const WtabArgs<NL> &, hipStream_t);
template <int NL> hipError_t hb_launch_wmac(const WmacArgs<NL> &, hipStream_t);

namespace {

thread_local std::string g_create_error;

struct DevBuf {
    void *p = nullptr;
    size_t n = 0;
    hipError_t ensure(size_t want) {
        if (want <= n) return hipSuccess;
        if (p) (void)hipFree(p);
        p = nullptr;
        n = 0;
        hipError_t e = hipMalloc(&p, want ? want : 1);
        if (e == hipSuccess) n = want;
        return e;
    }
    void release() {
        if (p) (void)hipFree(p);
        p = nullptr;
        n = 0;
    }
};

// Pinned host buffer (hipHostMalloc): async H2D staging.
struct HostBuf {
    void *p = nullptr;
    size_t n = 0;
    hipError_t ensure(size_t want) {
        if (want <= n) return hipSuccess;
        if (p) (void)hipHostFree(p);
        p = nullptr;
        n = 0;
        hipError_t e = hipHostMalloc(&p, want ? want : 1, 0);
        if (e == hipSuccess) n = want;
        return e;
    }
    void release() {
        if (p) (void)hipHostFree(p);
        p = nullptr;
        n = 0;
    }
};

}  // namespace

struct hb_ctx {
    int device = 0;
    int num_cus = 256;
    hipStream_t stream = nullptr, copy = nullptr;
    hipEvent_t k0 = nullptr, k1 = nullptr;
    // phase marks of a device-resident two-pass encode (hb_last_kernel_phases):
    // after the set-up kernels, after the first pass, after the retry pass
    hipEvent_t ph[3] = {nullptr, nullptr, nullptr};
    bool ph_valid = false;
    hipEvent_t copied[2] = {nullptr, nullptr}, done[2] = {nullptr, nullptr};
    u32 *t0 = nullptr;
    unsigned long long *queue = nullptr;   // 16 slots of HB_QSLOT counters
    DevBuf alpha_raw, alpha_mont, xs, vals, vals2, wts, idx, partials, sums, data[2], tags, blen, gtags;
    DevBuf pfx, retry;   // two-pass encode: CFB prefix image, retry list
    DevBuf afrag;        // MFMA MAC: digit fragments of alpha_j R mod p
    DevBuf ctl;          // wsum column counters + flags (zero between operations)
    DevBuf mseeds, moffs, mdig;   // Merkle chunk seeds, offsets, HMAC digests
    DevBuf gdev;         // device-resident prove: the challenged blocks and tags, gathered
    DevBuf facc;         // fused prove: per-column limb sums over workgroups (zero between operations)
    DevBuf gup;          // prove of a small host file: the file, uploaded whole
    DevBuf wpw;          // split wide-prime encode: 256^e mod p, e < ss (for wide_key)
    DevBuf wtab;         // its digit table (A fragments), kz, status word
    Limbs wide_key;      // p of wpw, then ss (wide_prep)
    HostBuf gstage[2];   // host-file prove: pinned gather buffers (blocks | tags), double-buffered
    HostBuf hscratch;    // pinned staging of the encode's small host round trips (alpha, MFMA tables)
    // the alpha D2H into hscratch done / the MFMA-table H2D out of it done
    // (not yet waited for: the next round trip must wait before reusing hscratch)
    hipEvent_t ev_alpha = nullptr, ev_h2d = nullptr;
    // split wide-prime encode: alpha's PRF, its Montgomery form and the digit
    // table run on `side` beside the prefix image and the PRF passes (which do
    // not read alpha); ev_side0 orders them after the stream's earlier work,
    // ev_side1 orders the MAC after them
    hipStream_t side = nullptr;
    hipEvent_t ev_side0 = nullptr, ev_side1 = nullptr;
    bool h2d_pending = false;
    bool alpha_pending = false;   // the alpha D2H into hscratch not yet waited for
    bool prove_dirty = false;   // a prove stopped between its launches: counters to clear
    bool verify_dirty = false;  // a fused verify did not complete: its slots and sums to clear
    bool ctl_dirty = false;     // a weighted sum did not complete: clear its counters
    u32 wsum_token = 0;         // completion token of the last hb_wsum_kernel launch
    // HB_ENABLE_TEST_SWITCHES=1 when the context was created: the A/B and test
    // switches (sw_env) are honoured; otherwise none is even read
    bool switches = false;
    u32 *hres = nullptr; // pinned host buffer of the wsum results (+ status, token)
    bool sums_in_hres = true;   // the last wsum wrote its results straight into hres
    // R^2 mod p (Montgomery conversion) of the last prime seen: ~10 us of host
    // big-integer work per call otherwise, on a prove's critical path
    Limbs r2_p, r2_val;
    size_t hres_n = 0;
    std::string err;
    double last_ms = 0.0;
    u32 last_launches = 0;
    bool sums_polled = false;   // the last sum was a fused prove's: finish_sums polls its token
    hipStream_t own_stream = nullptr;   // `stream` unless hb_ctx_set_stream gave another
    // an HB_ASYNC encode still running: its counters, and the status and tries
    // of the last one completed (hb_ctx_wait)
    bool pending = false;
    unsigned long long *pend_q0 = nullptr, *pend_q7 = nullptr;
    int pend_rc = 0;
    std::string pend_err;
    u64 pend_tries = 0;
};

namespace {

int fail(hb_ctx *c, int code, const std::string &msg) {
    if (c) c->err = msg;
    return code;
}

int hipfail(hb_ctx *c, hipError_t e, const char *what) {
    return fail(c, HB_EHIP, std::string(what) + ": " + hipGetErrorString(e));
}

#define HB_CHECK(expr, what)                         \
    do {                                             \
        hipError_t e_ = (expr);                      \
        if (e_ != hipSuccess) return hipfail(c, e_, what); \
    } while (0)

// ------------------------------------------------------------------ A/B and test switches
// Environment switches that change HOW a result is computed (never what):
// engine and MAC variants for same-box A/Bs, shrunken buffers that force the
// overflow / multi-batch paths in tests, phase tracing.  All are behind one
// gate, HB_ENABLE_TEST_SWITCHES=1, read once when a context is created, so a
// stray variable in a production environment cannot change the speed.
// (HB_GATHER_THREADS, a deployment knob, is not a test switch.)
bool switch_gate() {
    const char *g = getenv("HB_ENABLE_TEST_SWITCHES");
    return g && g[0] == '1' && g[1] == 0;
}

const char *sw_env(const hb_ctx *c, const char *name) {
    if (!c->switches) return nullptr;
    const char *v = getenv(name);
    return v && *v ? v : nullptr;
}

struct SwitchName {
    const char *env;
    u32 bit;
};
const SwitchName kSwitches[] = {
    {"HB_NO_QUAD", HB_SW_NO_QUAD},
    {"HB_NO_MFMA", HB_SW_NO_MFMA},
    {"HB_MFMA_SECTOR_LOADS", HB_SW_MFMA_SECTOR_LOADS},
    {"HB_MFMA_LINE32", HB_SW_MFMA_LINE32},
    {"HB_MFMA_MIN_S", HB_SW_MFMA_MIN_S},
    {"HB_TEST_NO_EARLY_LIST", HB_SW_NO_EARLY_LIST},
    {"HB_TEST_RETRY_CAP", HB_SW_RETRY_CAP},
    {"HB_TEST_PROVE_BATCH", HB_SW_PROVE_BATCH},
    {"HB_TRACE_PHASES", HB_SW_TRACE_PHASES},
    {"HB_HOST_WINDOW_MIB", HB_SW_HOST_WINDOWS},
    {"HB_HOST_AHEAD", HB_SW_HOST_WINDOWS},
    {"HB_NO_PROVE_GATHER", HB_SW_NO_PROVE_GATHER},
    {"HB_SUMS_ON_DEVICE", HB_SW_SUMS_ON_DEVICE},
    {"HB_NO_PROVE_PLACE", HB_SW_NO_PROVE_PLACE},
    {"HB_NO_PROVE_FUSE", HB_SW_NO_PROVE_FUSE},
    {"HB_SYNC_WAIT", HB_SW_SYNC_WAIT},
    {"HB_NO_VERIFY_FUSE", HB_SW_NO_VERIFY_FUSE},
    {"HB_NO_SMALL_ENCODE", HB_SW_NO_SMALL_ENCODE},
    {"HB_NO_PROVE_UPLOAD", HB_SW_NO_PROVE_UPLOAD},
    {"HB_MID_BLOCKS", HB_SW_MID_BLOCKS},
    {"HB_NO_WIDE", HB_SW_NO_WIDE},
    {"HB_WMAC_WPE", HB_SW_WMAC_WPE},
    {"HB_WIDE_SYNC_ALPHA", HB_SW_WIDE_SYNC_ALPHA},
    {"HB_QCHUNK", HB_SW_QCHUNK},
};

int nl_for_bits(int bits) {
    if (bits <= 64) return 2;
    if (bits <= 256) return 8;
    if (bits <= 512) return 16;
    if (bits <= 1024) return 32;
#if !defined(HB_NO_NL64)
    if (bits <= 2048) return 64;
#endif
    return 0;
}

template <int NL>
bool make_prf(const uint8_t *key, size_t key_len, const uint8_t *range_be, size_t range_len,
              PrfParams<NL> &P, int &nr) {
    AesKey k;
    if (!aes_expand(key, key_len, k)) return false;
    nr = k.nr;
    memset(&P, 0, sizeof P);
    memcpy(P.rk, k.rk, sizeof(u32) * 4 * (size_t)(k.nr + 1));
    aes_round1_zero_consts(k, P.r1z);
    Limbs R = from_be(range_be, range_len, NL);
    for (int t = 0; t < NL; ++t) P.R[t] = R[t];
    int bits = bitlen_be(range_be, range_len);
    P.nb = (u32)(bits + 7) / 8;
    P.topmask = (1u << (bits - 8 * ((int)P.nb - 1))) - 1u;
    return true;
}

template <int NL>
void make_mod(const Limbs &p, ModP<NL> &M) {
    memset(&M, 0, sizeof M);
    for (int t = 0; t < NL; ++t) M.p[t] = p[t];
    M.pinv = mont_pinv(p[0]);
    M.inv_scaled = inv_scaled(p);
}

// R^2 mod p for NL limbs (R = 2^(32 NL)), cached per context for the last p.
const Limbs &r2_of(hb_ctx *c, const Limbs &p, int nl) {
    if (c->r2_p != p || c->r2_val.size() != (size_t)nl) {
        c->r2_val = pow2_mod(64u * (unsigned)nl, p);
        c->r2_p = p;
    }
    return c->r2_val;
}

int engine_grid(hb_ctx *c, u64 njobs) {
    u64 g = (njobs + HB_ENGINE_WG - 1) / HB_ENGINE_WG;
    u64 cap = (u64)HB_ENGINE_WG_PER_CU * (u64)c->num_cus;
    if (g > cap) g = cap;
    return (int)(g ? g : 1);
}

// Latency-bound PRF launches (a few thousand evaluations: challenges, alpha,
// KeyedPRF batches): every CU, and 64-job queue refills so that the jobs
// spread over many waves instead of queueing behind a few (each eval is a
// serial CFB chain); large launches keep 256-job refills.
struct EngineShape {
    int grid;
    u64 chunk;
};
EngineShape small_engine(hb_ctx *c, u64 njobs) {
    const u64 waves = (u64)c->num_cus * (HB_ENGINE_WG / 64);
    if (njobs >= waves * HB_QUEUE_CHUNK) return {engine_grid(c, njobs), (u64)HB_QUEUE_CHUNK};
    u64 g = (njobs + 63) / 64;   // 64-job chunks: at most one workgroup (CU) each
    if (g > (u64)c->num_cus) g = (u64)c->num_cus;
    return {(int)(g ? g : 1), 64};
}

// Jobs per queue refill in the encode engines: 256 for primes up to 256
// bits; 64 for the wider ones, whose tries are 64-256 serial AES, so that a
// pass does not end on a few waves still holding a refill's worth of jobs
// (8 GiB, 256 -> 64: 1024-bit S = 10 336 -> 360, 512-bit 573 -> 602,
// 2048-bit 182 -> 195 GiB/s; 256-bit S = 16 within noise, 1,002 vs 987;
// profiles/r06/r6q).  $HB_QCHUNK=n (A/B): n, rounded up to a multiple of 64
// (HbPool hands a wave at most one refill per take, so a refill must cover
// all 64 lanes).
u64 encode_qchunk(hb_ctx *c, int nl) {
    const char *q = sw_env(c, "HB_QCHUNK");
    if (!q) return nl >= 16 ? 64 : HB_QUEUE_CHUNK;
    u64 n = strtoull(q, nullptr, 10);
    n = (n + 63) / 64 * 64;
    return n ? n : 64;
}

// The quad engine (one KeyedPRF evaluation per four lanes, hb_engine_quad)
// while four lanes per job still fit on the GPU at once: such launches are
// bound by their longest serial CFB chain, not by throughput.  Every CU, one
// job per quad per refill (16 per wave).
bool use_quad(hb_ctx *c, u64 njobs) {
    if (sw_env(c, "HB_NO_QUAD")) return false;   // A/B and parity tests: the lane engine
    return njobs > 0 && 4 * njobs <= (u64)c->num_cus * HB_ENGINE_WG;
}
EngineShape quad_engine(hb_ctx *c, u64 njobs) {
    u64 g = (njobs + 15) / 16;
    if (g > (u64)c->num_cus) g = (u64)c->num_cus;
    return {(int)(g ? g : 1), 16};
}

int check_key(hb_ctx *c, size_t key_len) {
    if (key_len != 16 && key_len != 24 && key_len != 32)
        return fail(c, HB_EINVAL, "AES key must be either 16, 24, or 32 bytes long");
    return 0;
}

// KeyedPRF(key, range).eval(x) for n inputs (xs device array or x0 + k),
// results as NL-limb little-endian values in out (device).
template <int NL>
int run_prf(hb_ctx *c, const uint8_t *key, size_t key_len, const uint8_t *range_be, size_t range_len,
            const u64 *xs_dev, u64 x0, u64 n, u32 *out_dev, int queue_slot, int mode = 0,
            const u32 *digs_dev = nullptr, hipStream_t st = nullptr) {
    if (!st) st = c->stream;
    PrfArgs<NL> A;
    int nr = 0;
    if (!make_prf<NL>(key, key_len, range_be, range_len, A.prf, nr))
        return fail(c, HB_EINVAL, "invalid PRF key");
    A.xs = xs_dev;
    A.digs = digs_dev;
    A.x0 = x0;
    A.n = n;
    A.out = out_dev;
    A.t0 = c->t0;
    A.queue = c->queue + HB_QSLOT * queue_slot;
    if (n == 0) return 0;
    const bool quad = mode == 0 && use_quad(c, n);
    const EngineShape es = quad ? quad_engine(c, n) : small_engine(c, n);
    A.qchunk = es.chunk;
    // quad waves placed by SIMD as in the prove (hb_prove_place; every quad
    // launch's waves fit: use_quad); $HB_NO_PROVE_PLACE: the job-queue race
    A.place = quad && !sw_env(c, "HB_NO_PROVE_PLACE") ? 1u : 0u;
    HB_CHECK(hipMemsetAsync(A.queue, 0, HB_QSLOT * sizeof(unsigned long long), st), "hipMemsetAsync");
    HB_CHECK(hb_launch_prf<NL>(A, nr, quad ? 3 : mode, es.grid, st), "hb_prf_kernel launch");
    return 0;
}

// After a synchronize: did any PRF launch abandon a job (queue slot [2])?
int check_prf_slots(hb_ctx *c) {
    unsigned long long q[16 * HB_QSLOT];
    HB_CHECK(hipMemcpy(q, c->queue, sizeof q, hipMemcpyDeviceToHost), "hipMemcpy(queue)");
    for (int s = 0; s < 16; ++s)
        if (q[s * HB_QSLOT + 2]) return fail(c, HB_EINVAL, "PRF rejection sampling did not terminate");
    return 0;
}

// in (n x NL limbs, device) -> in * R mod p (device)
template <int NL>
int run_mont(hb_ctx *c, const Limbs &p, const u32 *in, u32 *out, u64 n, hipStream_t st = nullptr) {
    if (!st) st = c->stream;
    if (n == 0) return 0;
    MontArgs<NL> A;
    make_mod<NL>(p, A.mod);
    const Limbs &r2 = r2_of(c, p, NL);
    for (int t = 0; t < NL; ++t) A.r2[t] = r2[t];
    A.in = in;
    A.out = out;
    A.n = n;
    HB_CHECK(hb_launch_mont<NL>(A, st), "hb_mont_kernel launch");
    return 0;
}

struct PrimeInfo {
    int bits = 0, nl = 0;
    u32 ss = 0, tw = 0;
};

int parse_prime(hb_ctx *c, const uint8_t *p_be, size_t p_len, PrimeInfo &pi) {
    if (!p_be || p_len == 0) return fail(c, HB_EINVAL, "prime is empty");
    pi.bits = bitlen_be(p_be, p_len);
    // sectorsize = bitlen(p) // 8 >= 1 (PySwizzle.py:255); smaller primes make
    // the reference's encode loop never terminate (read(0) is never short)
    if (pi.bits < 8) return fail(c, HB_EINVAL, "prime must be at least 2^7 (sector size >= 1 byte)");
    if (!(p_be[p_len - 1] & 1)) return fail(c, HB_EINVAL, "prime must be odd");
    pi.nl = nl_for_bits(pi.bits);
    if (!pi.nl) return fail(c, HB_EUNSUPPORTED, "primes above 2048 bits are not supported by this build");
    if (pi.nl < 8) pi.nl = 8;
    pi.ss = (u32)pi.bits / 8;
    pi.tw = (u32)(pi.bits + 7) / 8;
    return 0;
}

// Sectors are full limb width and every sector start is 16-byte aligned:
// the kernels' batched 16-byte load path (hb_lane.hpp, ALIGN = 16).
bool full16(const PrimeInfo &pi, int nl, u64 C, const void *base) {
    return pi.ss == 4u * (u32)nl && pi.ss % 16 == 0 && C % 16 == 0 && ((uintptr_t)base % 16) == 0;
}

// ------------------------------------------------------------------ prepare
// The HIP runtime loads a translation unit's code object (hb_kern_*.hip, up
// to ~3 MiB each) at the first launch of one of its kernels.  hb_ctx_prepare
// does that ahead of the first encode / prove with a prime of the given size:
// every launcher is called with hb_load_only set on this thread, which only
// loads the kernel (hb_kernels.hpp, HB_LAUNCH); the flag is cleared again on
// every exit path, so no real launch can be skipped.
struct HbLoadOnly {
    HbLoadOnly() { hb_load_only = true; }
    ~HbLoadOnly() { hb_load_only = false; }
};

template <int NL>
void prepare_nl(hb_ctx *c) {
    EncodeArgs<NL> E;
    memset(&E, 0, sizeof E);
    for (int pass = 0; pass <= 3; ++pass)
        for (int align : {16, 1}) (void)hb_launch_encode<NL>(E, 14, align, pass, 0, c->stream);
    if constexpr (NL >= 16) {   // the split wide-prime encode (wide_plan)
        for (int pass = 1; pass <= 3; ++pass) (void)hb_launch_encode<NL>(E, 14, 0, pass, 0, c->stream);
        WtabArgs<NL> WT;
        memset(&WT, 0, sizeof WT);
        (void)hb_launch_wtab<NL>(WT, c->stream);
        WmacArgs<NL> WM;
        memset(&WM, 0, sizeof WM);
        (void)hb_launch_wmac<NL>(WM, c->stream);
    }
    for (int align : {16, 1}) (void)hb_launch_mac<NL>(E, align, c->stream);
    Prf2Args<NL> P2;
    memset(&P2, 0, sizeof P2);
    (void)hb_launch_prf_pair<NL>(P2, 14, 0, c->stream);
    PrfArgs<NL> P;
    memset(&P, 0, sizeof P);
    for (int mode : {0, 3}) (void)hb_launch_prf<NL>(P, 14, mode, 0, c->stream);
    if constexpr (NL <= HB_FUSE_MAX_NL) {
        VerifyArgs<NL> VA;
        memset(&VA, 0, sizeof VA);
        (void)hb_launch_verify_fused<NL>(VA, 14, 0, c->stream);
    }
    MontArgs<NL> M;
    memset(&M, 0, sizeof M);
    (void)hb_launch_mont<NL>(M, c->stream);   // n = 0: grid 0
    WsumArgs<NL> W;
    memset(&W, 0, sizeof W);
    for (int align : {16, 1}) (void)hb_launch_wsum<NL>(W, align, 0, c->stream);
    ProveArgs<NL> V;
    memset(&V, 0, sizeof V);
    (void)hb_launch_prove_prf<NL>(V, 14, 3, 3, 0, c->stream);
    (void)hb_launch_prove_prf<NL>(V, 14, 0, 0, 0, c->stream);
}

// ------------------------------------------------------------------ encode
// Retry-list capacity for a launch of nb blocks: the first pass rejects each
// block with probability q = 1 - p / 2^bitlen(p); room for the mean plus 8
// standard deviations (a block that finds the list full is finished in place
// by the first-pass kernel, so the bound only affects speed, never results).
u64 retry_capacity(const hb_ctx *c, const uint8_t *p_be, size_t p_len, u64 nb) {
    size_t i = 0;
    while (i < p_len && p_be[i] == 0) ++i;
    u64 top = 0;
    size_t k = 0;
    for (; k < 8 && i + k < p_len; ++k) top = (top << 8) | p_be[i + k];
    const int rest = 8 * (int)(p_len - i - k);
    const double frac = ldexp((double)top, rest - bitlen_be(p_be, p_len));
    double q = 1.0 - frac;
    if (q < 0) q = 0;
    const double mean = q * (double)nb;
    double cap = mean + 8.0 * sqrt(mean) + 1024.0;
    // test hook: a smaller list, to exercise the in-place overflow path
    if (const char *t = sw_env(c, "HB_TEST_RETRY_CAP")) cap = fmin(cap, atof(t));
    return cap >= (double)nb ? nb : (u64)cap;
}

// Host-built inputs of the MFMA MAC (hb_kernels.hpp, hb_mfma_block_acc /
// hb_mfma16_block_acc) from alpha_j (c->alpha_raw, on the device): the
// A-operand fragments and kz.
//
// Dense (default): sector j = sum_k u_k 256^(31-k) (big-endian bytes u_k), so
//     alpha_j u_j = sum_k u_k r_jk (mod p),  r_jk = alpha_j 256^(31-k) mod p.
// Each r_jk is taken as the representative in [-0x8080..80, 0x7f7f..7f] (the
// range of 32 signed base-256 digits, width 2^256 - 1 >= p) and split into its
// digits D_jk[c], c < 32; the MFMA then computes, per block, the 32 column
// sums sum_jk D_jk[c] (u_jk - 128) (|.| <= S 2^19 < 2^31), and
//     T = sum_c col_c 256^c + kz,  kz = 128 sum_jk r_jk + p 2^w > 0
// is = sum_j alpha_j u_j (mod p) and < 2^282 (w below), so the finish is
// (T + F) mod p by one quotient-estimate reduction.  One tile row per output
// digit, every entry used.  HB_MAC_MONT (A/B variant): r_jk carries R
// (alpha_j R mod p, c->alpha_mont), w = 40, T < 2^297 and the finish is the
// REDC of T + F R.
// HB_MFMA_TOEPLITZ (A/B variant): the 33 balanced digits d_i of alpha_j R mod p
// as the Toeplitz band of the unreduced product (64 output digits, two tiles
// per sector, half of each zero), kz = Q sum_j alpha_j R mod p + p 2^268.
// Layouts: 1 = sector loads (slot j holds sector j: lane (h, m) byte e is
// byte 16 h + e of sector j); 2 = whole-line loads (S % 4 == 0; slot j0 + r,
// j0 % 4 == 0, holds chunk 4h + r of the line of sectors j0 .. j0+3: byte
// 16 (r % 2) + e of sector j0 + 2h + r / 2), see hb_line_loads; 3 = the
// 16x16x64 MFMA (S % 2 == 0, dense only), see hb_mfma16_block_acc.
// Two halves, so that the host builds the tables while the GPU runs the
// prefix kernel: mfma_tables_begin enqueues the D2H of alpha (after the
// alpha PRF, before the prefix kernel in stream order); mfma_tables waits for
// that copy only, builds the tables and enqueues their H2D (after the prefix
// kernel, before the first pass), without synchronizing the stream.
int mfma_tables_begin(hb_ctx *c, u32 S) {
    const int NL = 8;
    if (c->h2d_pending) {   // the previous call's H2D still reads hscratch
        HB_CHECK(hipEventSynchronize(c->ev_h2d), "H2D(afrag)");
        c->h2d_pending = false;
    }
    if (c->alpha_pending) {
        // an encode that failed between its alpha D2H and mfma_tables: that
        // copy may still be writing hscratch (error path only)
        HB_CHECK(hipStreamSynchronize(c->stream), "D2H(alpha)");
        c->alpha_pending = false;
    }
    HB_CHECK(c->hscratch.ensure((size_t)S * NL * 4 + (size_t)HB_MFMA_NT * S * 64 * 16), "hipHostMalloc(scratch)");
#if !defined(HB_MFMA_TOEPLITZ) && !defined(HB_MAC_MONT)
    // the dense tiles carry alpha_j itself (the finish adds F and reduces,
    // no REDC); HB_MAC_MONT / the Toeplitz MAC: alpha_j R mod p
    const void *asrc = c->alpha_raw.p;
#else
    const void *asrc = c->alpha_mont.p;
#endif
    HB_CHECK(hipMemcpyAsync(c->hscratch.p, asrc, (size_t)S * NL * 4, hipMemcpyDeviceToHost, c->stream), "D2H(alpha)");
    c->alpha_pending = true;   // until mfma_tables (or the next begin) waits for ev_alpha
    HB_CHECK(hipEventRecord(c->ev_alpha, c->stream), "hipEventRecord");
    return 0;
}

int mfma_tables(hb_ctx *c, const Limbs &p, u32 S, u32 kz[17], int layout) {
    const int NL = 8;
    u32 *am = (u32 *)c->hscratch.p;
    int8_t *frag = (int8_t *)c->hscratch.p + (size_t)S * NL * 4;
    const size_t frag_bytes = (size_t)HB_MFMA_NT * S * 64 * 16;
    HB_CHECK(hipEventSynchronize(c->ev_alpha), "alpha PRF");
    c->alpha_pending = false;
    // layouts 1, 2 (32x32x32 B operand): slot s, lane half h, byte e ->
    // (sector j, byte k of sector j)
    auto src_of = [&](u32 slot, int h, int e, u32 &j, int &k) {
        if (layout == 2) {
            const u32 r = slot & 3u;
            j = (slot & ~3u) + 2u * (u32)h + r / 2u;
            k = 16 * (int)(r & 1u) + e;
        } else {
            j = slot;
            k = 16 * h + e;
        }
    };
#if !defined(HB_MFMA_TOEPLITZ)
    // D[(j * 32 + k) * 32 + c]: digit c of r_jk
    std::vector<int8_t> D((size_t)S * 32 * 32);
    u64 acc[12] = {0};   // sum_jk (r_jk mod p), then kz
    u64 nneg = 0;        // representatives r_jk - p taken
    for (u32 j = 0; j < S; ++j) {
        u32 x[NL];
        for (int t = 0; t < NL; ++t) x[t] = am[(size_t)j * NL + t];
        for (int k = 31; k >= 0; --k) {
            if (k < 31) {
                // x = 256 x mod p: eight doublings, each reduced (x < p < 2^256)
                for (int b = 0; b < 8; ++b) {
                    u32 top = x[NL - 1] >> 31;
                    for (int t = NL - 1; t > 0; --t) x[t] = (x[t] << 1) | (x[t - 1] >> 31);
                    x[0] <<= 1;
                    bool ge = top != 0;
                    if (!ge) {
                        ge = true;
                        for (int t = NL - 1; t >= 0; --t)
                            if (x[t] != p[t]) {
                                ge = x[t] > p[t];
                                break;
                            }
                    }
                    if (ge) {
                        u64 br = 0;
                        for (int t = 0; t < NL; ++t) {
                            const u64 d = (u64)x[t] - p[t] - br;
                            x[t] = (u32)d;
                            br = (d >> 63) & 1u;
                        }
                    }
                }
            }
            u64 cy = 0;
            for (int t = 0; t < NL; ++t) {
                cy += acc[t] + x[t];
                acc[t] = (u32)cy;
                cy >>= 32;
            }
            for (int t = NL; t < 12 && cy; ++t) {
                cy += acc[t];
                acc[t] = (u32)cy;
                cy >>= 32;
            }
            // representative: r = x if x <= 0x7f..7f, else x - p (two's complement)
            bool big = false;
            for (int t = NL - 1; t >= 0; --t)
                if (x[t] != 0x7f7f7f7fu) {
                    big = x[t] > 0x7f7f7f7fu;
                    break;
                }
            u32 r[NL];
            u64 br = 0;
            for (int t = 0; t < NL; ++t) {
                const u64 d = (u64)x[t] - (big ? p[t] : 0u) - br;
                r[t] = (u32)d;
                br = (d >> 63) & 1u;
            }
            nneg += big ? 1u : 0u;
            int carry = 0;
            int8_t *d = &D[((size_t)j * 32 + (size_t)k) * 32];
            for (int i = 0; i < 32; ++i) {
                const int v = (int)((r[i / 4] >> (8 * (i % 4))) & 0xffu) + carry;
                carry = v >= 128 ? 1 : 0;
                d[i] = (int8_t)(v - 256 * carry);
            }
            // exact: the digits' carry out cancels the sign (0 for r >= 0, 1 for r < 0)
            if (carry != (big ? 1 : 0)) return fail(c, HB_EINVAL, "internal: MFMA digit range");
        }
    }
    // kz = 128 sum (r_jk mod p) + p (2^w - 128 nneg)   (nneg <= 32 S <= 2^16).
    // |sum_jk r_jk u_jk| < 32 S 255 2^255 < S 2^268 < p 2^w with
    // w = ceil(log2 S) + 14 (p > 2^255), so T = sum r u + p 2^w > 0; without
    // the Montgomery factor (HB_MAC_MONT off) T < 2^282 for S <= 2048 and the
    // finish is one hb_reduce_small; with it, w = 40 as before
    u64 sh = 0;
    for (int t = 0; t < 12; ++t) {   // acc *= 128
        const u64 v = (acc[t] << 7) | sh;
        sh = acc[t] >> 25;
        acc[t] = v & 0xffffffffull;
    }
#if defined(HB_MAC_MONT)
    const int w = 40;
#else
    int w = 14;
    while ((1u << (w - 14)) < S) ++w;
#endif
    const u64 mult = (1ull << w) - 128ull * nneg;
    const u64 mlo = mult & 0xffffffffull, mhi = mult >> 32;
    u64 cy = 0;
    for (int t = 0; t < 12; ++t) {
        const u64 plo = t < NL ? (u64)p[t] * mlo : 0u;                      // < 2^64
        const u64 phi = t >= 1 && t - 1 < NL ? (u64)p[t - 1] * mhi : 0u;   // < 2^40
        const unsigned __int128 s = (unsigned __int128)acc[t] + (plo & 0xffffffffull) + phi + cy;
        acc[t] = (u64)s & 0xffffffffull;
        cy = (u64)(s >> 32) + (plo >> 32);
    }
    for (int t = 0; t <= 2 * NL; ++t) kz[t] = t < 12 ? (u32)acc[t] : 0u;
    if (layout == 3) {
        // v_mfma_i32_16x16x64_i8 A operand, tile t of K slice p (sectors
        // 2p, 2p+1) at fragment 2p + t: lane (g, m) = (l >> 4, l & 15) byte e
        // is A[row 16 t + m][k = 16 g + e], k = byte k % 32 of sector 2p + k / 32
        for (u32 p = 0; p < S / 2; ++p)
            for (int t = 0; t < 2; ++t)
                for (int l = 0; l < 64; ++l)
                    for (int e = 0; e < 16; ++e) {
                        const int k = 16 * (l >> 4) + e;
                        const u32 j = 2 * p + (u32)(k / 32);
                        frag[((size_t)(2 * p + t) * 64 + l) * 16 + e] =
                            D[((size_t)j * 32 + (size_t)(k % 32)) * 32 + (size_t)(16 * t + (l & 15))];
                    }
    } else {
        for (u32 slot = 0; slot < S; ++slot)
            for (int l = 0; l < 64; ++l)
                for (int e = 0; e < 16; ++e) {
                    u32 j;
                    int k;
                    src_of(slot, l >> 5, e, j, k);
                    frag[((size_t)slot * 64 + l) * 16 + e] = D[((size_t)j * 32 + (size_t)k) * 32 + (l & 31)];
                }
    }
#else
    std::vector<int> digits((size_t)S * 33);
    Limbs sum(NL, 0);
    for (u32 j = 0; j < S; ++j) {
        const u32 *a = &am[(size_t)j * NL];
        Limbs aj(a, a + NL);
        sum = add_mod(sum, aj, p);
        // balanced base-256 digits: alpha = sum_i d_i 256^i, d_i in [-128, 127], i <= 32
        int *d = &digits[(size_t)j * 33];
        int carry = 0;
        for (int i = 0; i < 32; ++i) {
            int x = (int)((a[i / 4] >> (8 * (i % 4))) & 0xffu) + carry;
            carry = x >= 128 ? 1 : 0;
            d[i] = x - 256 * carry;
        }
        d[32] = carry;
    }
    for (u32 slot = 0; slot < S; ++slot)
        for (int t = 0; t < 2; ++t)
            for (int l = 0; l < 64; ++l)
                for (int e = 0; e < 16; ++e) {
                    u32 j;
                    int k;   // byte of sector j (weight 256^(31 - k))
                    src_of(slot, l >> 5, e, j, k);
                    const int col = 32 * t + (l & 31), i = col - 31 + k;
                    const int *d = &digits[(size_t)j * 33];
                    frag[(((size_t)t * S + slot) * 64 + l) * 16 + e] = (int8_t)(i >= 0 && i <= 32 ? d[i] : 0);
                }
    // Q = 0x80..80 (32 bytes): sum_j alpha_j u_j = sum_j alpha_j (u_j - Q) + Q sum_j alpha_j
    Limbs q(NL, 0x80808080u);
    Limbs k = mul_mod(mod_any(q, p), sum, p);
    // kz = k + p 2^268 (> every negative sum_c D_c 256^c: |.| < S 2^511 <= 2^522)
    u64 carry = 0;
    for (int t = 0; t <= 2 * NL; ++t) {
        // p << 268: limb t gets bits from p limbs t - 8 (shift 12 within)
        u64 ps = 0;
        const int src = t - 8;
        if (src >= 0 && src < NL) ps |= (u64)p[src] << 12;
        if (src - 1 >= 0 && src - 1 < NL) ps |= (u64)p[src - 1] >> 20;
        ps &= 0xffffffffull;
        carry += ps + (t < NL ? k[t] : 0u);
        kz[t] = (u32)carry;
        carry >>= 32;
    }
#endif
    HB_CHECK(c->afrag.ensure(frag_bytes), "hipMalloc(afrag)");
    HB_CHECK(hipMemcpyAsync(c->afrag.p, frag, frag_bytes, hipMemcpyHostToDevice, c->stream), "H2D(afrag)");
    HB_CHECK(hipEventRecord(c->ev_h2d, c->stream), "hipEventRecord");
    c->h2d_pending = true;
    return 0;
}

// HB_HOST_REGISTER: host bytes page-locked by the library itself, in
// page-aligned windows of kWindow bytes -- the file read-only
// (hipHostRegisterReadOnly: a PROT_READ file mapping cannot be registered for
// writing), the tags for writing.  A helper thread registers up to kAhead
// windows ahead of the chunk being copied -- the page pinning overlaps the
// DMA of the previous window -- and unregisters each window once the
// copy-stream event recorded after its last chunk has completed, so at most
// about kAhead + 2 windows are pinned at a time.  Only pages lying wholly
// inside the buffer are registered: the partial pages at its two ends (which
// the neighbouring shard of a multi-device encode, or the caller, may own)
// are copied unpinned, and every copy is split so that no piece starts in a
// pinned range and runs past it.  A window whose registration fails (e.g.
// memory the caller registered already) is copied as is.  The reference
// reads the file through Python read() calls (PySwizzle.py:299;
// cxx/PythonSeekableFile.hxx:47-54); this is the replacement's staging.
struct HostWindows {
    u64 kWindow = 256ull << 20;   // $HB_HOST_WINDOW_MIB (test switch, A/B)
    u64 kAhead = 2;               // $HB_HOST_AHEAD (test switch, A/B)
    enum { NONE = 0, PINNED, UNPINNED, RECORDED, DONE };
    hb_ctx *c;
    unsigned int reg_flags;
    uintptr_t base = 0, end = 0;  // the whole pages inside the buffer
    u64 nwin = 0;
    std::vector<int> state;
    std::vector<hipEvent_t> ev;
    std::mutex m;
    std::condition_variable cv;
    u64 allowed = 0;        // windows [0, allowed) may be registered
    u64 next_reg = 0;       // next window the helper registers
    u64 next_rec = 0;       // next window the main thread records an event for
    bool quit = false;
    std::thread th;

    // host bytes [p, p + len); read_only: the device only reads them (the
    // file), else it writes them (the tags); scale: window size relative to
    // the file's (the tags of a file window: tw / C of it, so that the first
    // tag copy waits for a small window only)
    HostWindows(hb_ctx *ctx, const void *p, u64 len, bool read_only, double scale = 1.0)
        : c(ctx), reg_flags(read_only ? hipHostRegisterReadOnly : hipHostRegisterDefault) {
        if (const char *v = sw_env(c, "HB_HOST_WINDOW_MIB")) kWindow = (u64)(atoi(v) > 0 ? atoi(v) : 256) << 20;
        if (const char *v = sw_env(c, "HB_HOST_AHEAD")) kAhead = (u64)(atoi(v) > 0 ? atoi(v) : 2);
        kWindow = ((u64)((double)kWindow * scale) + 4095) & ~(u64)4095;
        if (kWindow < (2ull << 20)) kWindow = 2ull << 20;
        base = ((uintptr_t)p + 4095) & ~(uintptr_t)4095;
        end = ((uintptr_t)p + len) & ~(uintptr_t)4095;
        nwin = end > base ? (end - base + kWindow - 1) / kWindow : 0;
        if (!nwin) end = base;
        state.assign((size_t)nwin, NONE);
        ev.assign((size_t)nwin, nullptr);
        allowed = kAhead + 1;   // start pinning right away, ahead of the first copy
        th = std::thread([this] { run(); });
    }
    ~HostWindows() { finish(); }
    u64 window_of(uintptr_t a) const { return (u64)((a - base) / kWindow); }
    uintptr_t wlo(u64 w) const { return base + w * kWindow; }
    uintptr_t whi(u64 w) const { return base + (w + 1) * kWindow < end ? base + (w + 1) * kWindow : end; }

    void run() {
        (void)hipSetDevice(c->device);
        std::unique_lock<std::mutex> lk(m);
        for (;;) {
            if (next_reg < nwin && next_reg < allowed && !quit) {
                const u64 w = next_reg;
                lk.unlock();
                const hipError_t e = hipHostRegister((void *)wlo(w), (size_t)(whi(w) - wlo(w)), reg_flags);
                if (e != hipSuccess) (void)hipGetLastError();
                lk.lock();
                state[(size_t)w] = e == hipSuccess ? (int)PINNED : (int)UNPINNED;
                ++next_reg;
                cv.notify_all();
                continue;
            }
            // a window whose last copy is enqueued: unpin it once that copy is done
            u64 u = nwin;
            for (u64 k = 0; k < nwin; ++k)
                if (state[(size_t)k] == RECORDED) { u = k; break; }
            if (u < nwin) {
                lk.unlock();
                (void)hipEventSynchronize(ev[(size_t)u]);
                (void)hipHostUnregister((void *)wlo(u));
                lk.lock();
                state[(size_t)u] = DONE;
                cv.notify_all();
                continue;
            }
            if (quit) return;
            cv.wait(lk);
        }
    }
    // wait until the windows overlapping [a, b) are settled (registered or
    // failed), allowing registration kAhead windows further
    void acquire(uintptr_t a, uintptr_t b) {
        const uintptr_t lo = a > base ? a : base, hi = b < end ? b : end;
        if (hi <= lo) return;
        const u64 wb = window_of(hi - 1);
        std::unique_lock<std::mutex> lk(m);
        if (wb + 1 + kAhead > allowed) {
            allowed = wb + 1 + kAhead;
            cv.notify_all();
        }
        cv.wait(lk, [&] { return next_reg > wb; });
    }
    // every window wholly below address a is copied for good: record an event
    // on the copy stream behind those copies, for the helper to unpin it
    void release_below(uintptr_t a) {
        const u64 wa = a >= end ? nwin : a <= base ? 0 : window_of(a);
        while (next_rec < wa) {
            const u64 w = next_rec++;
            std::unique_lock<std::mutex> lk(m);
            if (state[(size_t)w] != PINNED) {
                if (state[(size_t)w] == UNPINNED) state[(size_t)w] = DONE;
                continue;
            }
            lk.unlock();
            hipEvent_t e = nullptr;
            if (hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess ||
                hipEventRecord(e, c->copy) != hipSuccess) {
                if (e) (void)hipEventDestroy(e);
                (void)hipStreamSynchronize(c->copy);
                e = nullptr;
            }
            lk.lock();
            ev[(size_t)w] = e;
            if (e) state[(size_t)w] = RECORDED;
            else {
                (void)hipHostUnregister((void *)wlo(w));
                state[(size_t)w] = DONE;
            }
            cv.notify_all();
        }
    }
    // enqueue the copy of host bytes [a, e) to (h2d) or from the device
    // memory at dev on the copy stream: one piece per window, the partial
    // end pages unpinned; windows wholly behind e are handed to the helper
    hipError_t copy(void *dev, uintptr_t a, uintptr_t e, bool h2d) {
        acquire(a, e);
        for (uintptr_t x = a; x < e;) {
            uintptr_t y = e;
            if (x < base) y = base < e ? base : e;
            else if (x < end) y = whi(window_of(x)) < e ? whi(window_of(x)) : e;
            uint8_t *d = (uint8_t *)dev + (x - a);
            const hipError_t r = h2d ? hipMemcpyAsync(d, (const void *)x, (size_t)(y - x), hipMemcpyHostToDevice, c->copy)
                                     : hipMemcpyAsync((void *)x, d, (size_t)(y - x), hipMemcpyDeviceToHost, c->copy);
            if (r != hipSuccess) return r;
            x = y;
        }
        release_below(e);
        return hipSuccess;
    }
    // stop the helper; every window still pinned is unpinned after the copy
    // stream has drained (all exit paths, errors included)
    void finish() {
        if (!th.joinable()) return;
        {
            std::lock_guard<std::mutex> lk(m);
            quit = true;
            cv.notify_all();
        }
        th.join();
        bool any = false;
        for (u64 w = 0; w < nwin; ++w) any = any || state[(size_t)w] == PINNED || state[(size_t)w] == RECORDED;
        if (any) (void)hipStreamSynchronize(c->copy);
        for (u64 w = 0; w < nwin; ++w) {
            if (state[(size_t)w] == PINNED || state[(size_t)w] == RECORDED) (void)hipHostUnregister((void *)wlo(w));
            if (ev[(size_t)w]) (void)hipEventDestroy(ev[(size_t)w]);
            ev[(size_t)w] = nullptr;
            state[(size_t)w] = DONE;
        }
    }
};

// Complete an HB_ASYNC encode: wait for its kernels, read its PRF counters;
// the status is kept for hb_ctx_wait.  Every other entry point settles first
// (its own kernels would reuse the counters and scratch buffers).
void settle(hb_ctx *c) {
    if (!c->pending) return;
    c->pending = false;
    const std::string keep = c->err;
    // the FIRST failure since the last hb_ctx_wait is kept: a second async
    // encode issued before the wait must not hide the first one's error
    auto done = [&](int rc) {
        if (rc && c->pend_rc == 0) {
            c->pend_rc = rc;
            c->pend_err = c->err;
        }
        c->err = keep;
    };
    float ms = 0.f;
    unsigned long long q[HB_QSLOT], r[HB_QSLOT];
    hipError_t e = hipEventSynchronize(c->k1);
    if (e == hipSuccess) e = hipEventElapsedTime(&ms, c->k0, c->k1);
    if (e == hipSuccess) e = hipMemcpy(q, c->pend_q0, sizeof q, hipMemcpyDeviceToHost);
    if (e == hipSuccess) e = hipMemcpy(r, c->pend_q7, sizeof r, hipMemcpyDeviceToHost);
    if (e != hipSuccess) return done(hipfail(c, e, "async encode"));
    c->last_ms = ms;
    if (q[2] || r[2]) return done(fail(c, HB_EINVAL, "PRF rejection sampling did not terminate for some blocks"));
    c->pend_tries += q[1] + r[1];
    done(check_prf_slots(c));
}

// ------------------------------------------------------------------ split wide-prime encode
// Primes above 256 bits (NL >= 16), PySwizzle PRF, two-pass: the first-try
// and retry passes store F only (ALIGN = 0, 1,024-thread workgroups), and the
// sector MAC runs on the int8 matrix cores (hb_wide.hpp): a digit table built
// on the device from alpha (hb_wtab_kernel), then per launch hb_wmac_kernel
// (whole blocks) and hb_wmac_tail_kernel (the short last block, VALU).
// Applies when C % 16 == 0 (16-byte block loads), C <= HB_WIDE_MAX_C and w
// (below) <= 29; $HB_NO_WIDE (test switch, A/B): the in-kernel VALU MAC.
//
// w: the smallest shift with p 2^w > C 128 2^(8D - 1) >= |sum_x r'_x (u_x -
// 128)| (|r'_x| <= 2^(8D-1)), so that T = sum_c col_c 256^c + kz > 0; then
// T < 3 p 2^w and T + F < 2^32 p, the range of hb_reduce_small; the column
// sums |col_c| <= C 2^14 stay inside int32 for C <= HB_WIDE_MAX_C.
template <int NL>
bool wide_plan(const PrimeInfo &pi, u64 C, WtabArgs<NL> &W, u32 &w_out) {
    if (C == 0 || C % 16 != 0 || C > HB_WIDE_MAX_C) return false;
    const u32 D = pi.tw;
    int lc = 0;
    while ((1ull << lc) < C) ++lc;   // ceil(log2 C)
    const int w = lc + 8 * (int)D + 7 - pi.bits;
    if (w < 0 || w > 29) return false;
    W.C = (u32)C;
    W.ss = pi.ss;
    W.D = D;
    W.Mt = (D + 15) / 16;
    W.nslices = (u32)((C + 63) / 64);
    if ((int)W.Mt > NL / 4) return false;
    for (int t = 0; t < NL; ++t) W.half[t] = 0;
    for (u32 i = 0; i < D; ++i) W.half[i / 4] |= 0x7fu << (8 * (i % 4));
    w_out = (u32)w;
    return true;
}

// The tables of wide_plan that depend on p and ss only -- 256^e mod p (e <
// ss, uploaded to c->wpw) and 128 G mod p, G = sum_e 256^e -- rebuilt when p
// or ss changes; p 2^w into W.p2w.
template <int NL>
int wide_prep(hb_ctx *c, const Limbs &p, const PrimeInfo &pi, u32 w, WtabArgs<NL> &W) {
    Limbs key(p);
    key.push_back(pi.ss);
    if (key != c->wide_key) {
        std::vector<u32> pw((size_t)pi.ss * NL, 0);
        Limbs x(NL, 0), g(NL, 0);
        x[0] = 1;
        if (cmp(x, p) >= 0) x = mod_any(x, p);
        for (u32 e = 0; e < pi.ss; ++e) {
            for (int t = 0; t < NL; ++t) pw[(size_t)e * NL + t] = x[t];
            g = add_mod(g, x, p);
            for (int b = 0; b < 8; ++b) x = add_mod(x, x, p);   // x = 256 x mod p
        }
        for (int b = 0; b < 7; ++b) g = add_mod(g, g, p);       // 128 G mod p
        HB_CHECK(c->wpw.ensure(pw.size() * 4), "hipMalloc(wide pw)");
        HB_CHECK(hipStreamSynchronize(c->stream), "hipStreamSynchronize");   // an earlier table build may read wpw
        HB_CHECK(hipMemcpy(c->wpw.p, pw.data(), pw.size() * 4, hipMemcpyHostToDevice), "H2D(wide pw)");
        c->wide_key = key;
        c->wide_key.insert(c->wide_key.end(), g.begin(), g.end());   // cached 128 G mod p
    }
    for (int t = 0; t < NL; ++t) W.g128[t] = c->wide_key[c->wide_key.size() - NL + t];
    // p 2^w, NL + 1 limbs
    for (int t = 0; t <= NL; ++t) {
        const u64 lo = t < NL ? (u64)p[t] << w : 0u;
        const u64 hi = t >= 1 && w ? (u64)p[t - 1] >> (32 - w) : 0u;
        W.p2w[t] = (u32)(lo | hi);
    }
    W.pw = (const u32 *)c->wpw.p;
    return 0;
}

template <int NL>
int encode_impl(hb_ctx *c, const uint8_t *p_be, size_t p_len, const PrimeInfo &pi, u32 S,
                const uint8_t *f_key, const uint8_t *a_key, size_t key_len, u64 block_base,
                const uint8_t *data, u64 len, u64 nblocks, uint8_t *tags, u32 flags, u64 *tries_out) {
    Limbs p = from_be(p_be, p_len, NL);
    const u64 C = (u64)pi.ss * S;
    // $HB_TRACE_PHASES: host-side phase times of this call on stderr (the
    // stream is synchronized at each mark; diagnosis of first-call costs)
    const bool trace = sw_env(c, "HB_TRACE_PHASES") != nullptr;
    const auto t_start = std::chrono::steady_clock::now();
    auto mark = [&](const char *what) {
        if (!trace) return;
        (void)hipStreamSynchronize(c->stream);
        fprintf(stderr, "[hb_encode] %-28s %9.3f ms\n", what,
                std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t_start).count());
    };
    // the side stream's work of an earlier split encode reads the alpha and
    // table buffers regrown below; it has finished unless that call failed
    // between its launches (the MAC waits for it otherwise)
    HB_CHECK(hipStreamSynchronize(c->side), "hipStreamSynchronize(side)");
    // alpha_j R mod p, j < S  (alpha = KeyedPRF(alpha_key, p), PySwizzle.py:291,302)
    HB_CHECK(c->alpha_raw.ensure((size_t)S * NL * 4), "hipMalloc");
    HB_CHECK(c->alpha_mont.ensure((size_t)S * NL * 4), "hipMalloc");
    mark("alpha buffers");
    const bool cxx = flags & HB_PRF_CXX;
    if (cxx && (pi.tw % 16 != 0 || pi.tw > 4u * NL))
        return fail(c, HB_EUNSUPPORTED, "cxx prf mode needs ByteCount(p) to be a multiple of 16");
    // Small inputs -- as many blocks per launch as the quad engine runs at once
    // (use_quad): one placed quad-engine launch for the blocks' F and the
    // sectors' alpha (hb_prf_pair_kernel) + hb_mac_kernel, no prefix image
    // and no retry pass ($HB_NO_SMALL_ENCODE, test switch: the two-pass
    // engine for every size).
    const u64 cb0 = C ? ((256ull << 20) / C ? (256ull << 20) / C : 1) : 1;
    const u64 launch_max = (flags & HB_DATA_ON_DEVICE) ? nblocks : (nblocks < cb0 ? nblocks : cb0);
    // Mid-size inputs (up to 17 x 256 x #CUs blocks per launch: 1,114,112 on
    // MI355X, so that 2^20 + 1 blocks qualify): the same two launches with
    // the quad engine on a job queue instead of placed waves -- quads refill
    // as their jobs finish, the launch's longest rejection chain runs at the
    // quad engine's round latency instead of a lone lane's, and there is no
    // prefix image or retry list.  Benchmark prime P256, S = 16: 64 MiB 0.42
    // vs 1.18 ms, 256 MiB 0.88 vs 1.48, 512 MiB (2^20 + 1 blocks) 1.50 vs
    // 1.63; S = 1, 2^20 + 1 blocks 1.07 vs 1.58; 1024-bit S = 10, 839 K
    // blocks 6.54 vs 8.75; but a 256-bit prime with E[tries] 1.95 at 2 M
    // blocks 3.58 vs 3.32 (profiles/r05/mid).  Wider primes keep the
    // advantage longer (their two-pass retry chains are 2-4x longer): up to
    // 32 x 256 x #CUs blocks for NL >= 16 -- 512-bit S = 16, 2^20 + 1 blocks
    // 3.73 vs 5.01 ms; 1024-bit S = 10, 1.68 M blocks 11.0 vs 11.6, but 2.5 M
    // 15.7 vs 15.3 (profiles/r05/mid/wide_*.log).  Round 6 gave both paths
    // of the wide primes the MFMA MAC (hb_wmac_kernel): mid vs two-pass
    // 1024-bit S = 10 1 GiB 4.83 vs 6.73 ms, 2 GiB 7.92 vs 8.32; 512-bit
    // S = 16 1.2 GiB 3.22 vs 3.72; 2048-bit S = 4 1 GiB 7.20 vs 8.82
    // (profiles/r06/r6j) -- fits of both (mid ~ 4.7 / 2.6 / 6.9 ms per M
    // blocks, two-pass ~ 4.1 / 2.0 / 4.0 ms + 2.8 / 1.3 / 4.6 per M) cross
    // at 2.2 / 1.6 / 1.7 M blocks, next to the 2.1 M bound of then.  The
    // 64-job refills and the coalesced MAC finish sped the two-pass engine up
    // more: mid vs two-pass 1024-bit 1 GiB 202 vs 200 GiB/s, 1.5 GiB 237 vs
    // 246, 2 GiB 258 vs 277; 512-bit 1 GiB 334 vs 340, 2 GiB 453 vs 455;
    // 2048-bit 1 and 2 GiB equal (profiles/r06/r6aa) -- so the bound for
    // NL >= 16 is now 16 x 256 x #CUs (1 M blocks).
    // $HB_MID_BLOCKS (test switch, A/B): another bound, 0 = none.
    const char *mid_env = sw_env(c, "HB_MID_BLOCKS");
    const u64 mid_max = mid_env ? strtoull(mid_env, nullptr, 10) : (NL <= 8 ? 17ull : 16ull) * 256ull * (u64)c->num_cus;
    const bool small = !cxx && !(flags & HB_ENCODE_SINGLE_PASS) && launch_max &&
                       (use_quad(c, launch_max + S) || launch_max <= mid_max) && !sw_env(c, "HB_NO_SMALL_ENCODE");
    int rc = 0;

    EncodeArgs<NL> A;
    memset(&A, 0, sizeof A);
    A.qchunk = encode_qchunk(c, NL);
    int mf_layout = 0;   // MFMA MAC table layout (0: VALU MAC)
    if constexpr (NL == 8) {
        // MFMA MAC tables (hb_mfma_block_acc): 256-bit primes with whole
        // 32-byte sectors, PySwizzle PRF, two-pass encode
        // (below 4 sectors per block the VALU MAC is cheaper than the MFMA
        // phase's fixed cost: at configs[1], S = 1, the m16 MFMA MAC measured
        // 70.98 vs 71.32 GiB/s, same-box A/B, profiles/r04/l)
        // $HB_MFMA_MIN_S: the smallest sector count given the MFMA MAC (A/B,
        // read per call like every switch)
        const char *ms = sw_env(c, "HB_MFMA_MIN_S");
        const u32 min_s = ms ? (u32)atoi(ms) : 4u;
        if (!cxx && !small && pi.ss == 32 && S >= min_s && S <= HB_MFMA_MAX_S && !(flags & HB_ENCODE_SINGLE_PASS) &&
            !sw_env(c, "HB_NO_MFMA")) {
            // 3: the 16x16x64 MFMA, whose B operand is the whole-line load
            // shape (S even); 2: 32x32x32 with whole-line loads and an
            // in-quad transpose (S % 4 == 0; $HB_MFMA_LINE32, A/B); 1:
            // 32x32x32 with sector-shaped loads ($HB_MFMA_SECTOR_LOADS, A/B)
#if defined(HB_NO_LINE_LOADS)
            const int layout = 1;
#else
            const bool sector = sw_env(c, "HB_MFMA_SECTOR_LOADS") != nullptr;
#if defined(HB_MFMA_TOEPLITZ)
            const bool m16 = false;
#else
            const bool m16 = S % 2 == 0 && !sector && !sw_env(c, "HB_MFMA_LINE32");
#endif
            const int layout = m16 ? 3 : S % 4 == 0 && !sector ? 2 : 1;
#endif
            mf_layout = layout;   // tables: mfma_tables_begin / mfma_tables below
        }
    }
    int nr = 0;
    if (!make_prf<NL>(f_key, key_len, p_be, p_len, A.prf, nr)) return fail(c, HB_EINVAL, "invalid key");
    make_mod<NL>(p, A.mod);
    if (A.prf.nb >= 4) A.rtop = hb_range_top<NL>(A.prf);
    // test hook: no early retry listing (every rejected first try is listed
    // after the try without its digest, and the retry pass hashes the index)
    if (sw_env(c, "HB_TEST_NO_EARLY_LIST")) A.rtop = 0xffffffffu;
    A.alpha_mont = (const u32 *)c->alpha_mont.p;
    A.t0 = c->t0;
    A.C = C;
    A.tw = pi.tw;
    A.ss = pi.ss;
    A.S = S;
    unsigned long long *q0 = c->queue, *q7 = c->queue + HB_QSLOT * HB_SLOT_RETRY;
    // slots 0 (first pass / small-input F) and 1 (alpha)
    HB_CHECK(hipMemsetAsync(q0, 0, 2 * HB_QSLOT * sizeof(unsigned long long), c->stream), "hipMemsetAsync");
    HB_CHECK(hipMemsetAsync(q7, 0, HB_QSLOT * sizeof(unsigned long long), c->stream), "hipMemsetAsync");

    const bool tags_dev = flags & HB_TAGS_ON_DEVICE;
    const bool data_dev = flags & HB_DATA_ON_DEVICE;
    uint8_t *dtags = tags;
    if (!tags_dev) {
        HB_CHECK(c->tags.ensure((size_t)(nblocks * pi.tw)), "hipMalloc(tags)");
        dtags = (uint8_t *)c->tags.p;
    }
    // Host bytes go through the GPU in chunks of cb whole blocks.
    u64 cb = C ? (256ull << 20) / C : 1;
    if (cb < 1) cb = 1;
    const u64 launch_blocks = data_dev ? nblocks : (nblocks < cb ? nblocks : cb);
    // two passes (first tries with the prefix image, then the retry list) for
    // PySwizzle; the cxx prf (2 AES per try, no prefix) runs single-pass: a
    // cxx two-pass variant with the MFMA MAC measured 1,799 vs 2,246 GiB/s
    // (profiles/r02/s8)
    const bool two_pass = !cxx && !small && A.prf.nb >= 4 && !(flags & HB_ENCODE_SINGLE_PASS);
    if (small) {
        HB_CHECK(c->vals.ensure((size_t)launch_blocks * NL * 4), "hipMalloc(F)");
        A.fv = (const u32 *)c->vals.p;
    }
    // split wide-prime MAC (wide_plan), two-pass or small / mid-size inputs:
    // the two-pass F into the tag slots when they are exactly NL limbs wide
    // and 16-byte aligned, else into c->vals (the small path's F is there)
    WtabArgs<NL> WT;
    memset(&WT, 0, sizeof WT);
    bool wide = false;
    bool f_in_tags = false;
    if constexpr (NL >= 16) {
        u32 w = 0;
        // (the cxx prf: its single-pass engine, F-only as well)
        wide = (two_pass || small || (cxx && !(flags & HB_ENCODE_SINGLE_PASS))) &&
               (!data_dev || (uintptr_t)data % 16 == 0) && wide_plan<NL>(pi, C, WT, w) && !sw_env(c, "HB_NO_WIDE");
        if (wide) {
            if (int rc2 = wide_prep<NL>(c, p, pi, w, WT)) return rc2;
            const size_t fbytes = (size_t)WT.nslices * WT.Mt * 64 * 16;
            HB_CHECK(c->wtab.ensure(fbytes + (size_t)(NL + 1) * 4 + 16), "hipMalloc(wide table)");
            WT.mod = A.mod;
            WT.S = S;
            WT.alpha_mont = (const u32 *)c->alpha_mont.p;
            WT.afrag = (int8_t *)c->wtab.p;
            WT.kz = (u32 *)((uint8_t *)c->wtab.p + fbytes);
            WT.status = (unsigned int *)(WT.kz + NL + 1);
            f_in_tags = !small && pi.tw == 4u * NL && (uintptr_t)dtags % 16 == 0;
            if (!f_in_tags) HB_CHECK(c->vals.ensure((size_t)launch_blocks * NL * 4), "hipMalloc(F)");
            mark("wide tables");
        }
    }
    // alpha_j R mod p (large inputs; the small path's first launch computes
    // it): on the compute stream, or for the split wide-prime encode on the
    // side stream together with the digit table (wide_table below)
    const bool side = !small && wide && !sw_env(c, "HB_WIDE_SYNC_ALPHA");
    hipStream_t ast = side ? c->side : c->stream;
    if (side) {
        HB_CHECK(hipEventRecord(c->ev_side0, c->stream), "hipEventRecord");
        HB_CHECK(hipStreamWaitEvent(c->side, c->ev_side0, 0), "hipStreamWaitEvent");
    }
    if (!small) {
        rc = run_prf<NL>(c, a_key, key_len, p_be, p_len, nullptr, 0, S, (u32 *)c->alpha_raw.p, 1, cxx ? 1 : 0,
                         nullptr, ast);
        if (rc) return rc;
        mark("alpha PRF");
        rc = run_mont<NL>(c, p, (const u32 *)c->alpha_raw.p, (u32 *)c->alpha_mont.p, S, ast);
        if (rc) return rc;
        mark("alpha PRF + Montgomery");
    }
    if (two_pass) {
        A.retry_cap = retry_capacity(c, p_be, p_len, launch_blocks);
        HB_CHECK(c->retry.ensure((size_t)(A.retry_cap ? A.retry_cap : 1) * sizeof(HbRetry)), "hipMalloc(retry)");
        A.retry = (HbRetry *)c->retry.p;
        A.retry_count = q0 + 3;
        mark("retry list");
    }
    if (two_pass && !cxx) {
        HB_CHECK(c->pfx.ensure(HB_PFX_BYTES), "hipMalloc(prefix)");
        A.pfx = (const unsigned char *)c->pfx.p;
        AesKey k;
        aes_expand(f_key, key_len, k);
        uint8_t zero[16] = {0}, o[16];
        aes_encrypt_block(k, zero, o);
        A.o0 = o[0];
        mark("prefix image buffer");
    }
    if (mf_layout) {
        // every argument check and allocation is behind us: the alpha D2H
        // into hscratch starts here (mfma_tables waits for it)
        rc = mfma_tables_begin(c, S);
        if (rc) return rc;
    }
    c->last_launches = 0;
    c->ph_valid = false;
    float ms_total = 0.f;
    // the prefix image is part of the encode (rebuilt for every f_key): timed
    HB_CHECK(hipEventRecord(c->k0, c->stream), "hipEventRecord");
    if (two_pass && !cxx) {
        PrefixArgs PA;
        memcpy(PA.rk, A.prf.rk, sizeof PA.rk);
        PA.t0 = c->t0;
        PA.out = (unsigned char *)c->pfx.p;
        HB_CHECK(hb_launch_prefix(PA, nr, c->num_cus, c->stream), "hb_prefix_kernel launch");
        c->last_launches++;
    }
    // the digit table and kz from alpha_j R mod p (on the device, in stream
    // order): here for the two-pass encode, after the first PRF launch for
    // the small path (whose alpha that launch computes)
    bool wtab_pending = wide;
    auto wide_table = [&]() -> int {
        if constexpr (NL >= 16) {
            if (wtab_pending) {
                HB_CHECK(hipMemsetAsync(WT.status, 0, 4, ast), "hipMemsetAsync");
                HB_CHECK(hb_launch_wtab<NL>(WT, ast), "hb_wtab_kernel launch");
                if (side) HB_CHECK(hipEventRecord(c->ev_side1, c->side), "hipEventRecord");
                c->last_launches++;
                wtab_pending = false;
            }
        }
        return 0;
    };
    // tag = (F + sum_j alpha_j m_j) mod p of a launch's blocks from their F
    // (fsrc): hb_wmac_kernel for the whole blocks, the sector-parallel MAC
    // kernel for the short last one (and any past the end of the data)
    // (cxx: blocks without a sector read hold their final tag already, F
    // unreduced, from the PRF kernel -- the MAC kernels stop before them)
    auto wide_mac = [&](const uint8_t *d, u64 dlen, u64 nb, uint8_t *tg, const u32 *fsrc, int align) -> int {
        if constexpr (NL >= 16) {
            WmacArgs<NL> M;
            memset(&M, 0, sizeof M);
            M.mod = A.mod;
            M.data = d;
            M.len = dlen;
            M.nfull = dlen / C < nb ? dlen / C : nb;
            M.C = C;
            M.ss = pi.ss;
            M.S = S;
            M.tw = pi.tw;
            M.Mt = WT.Mt;
            M.nslices = WT.nslices;
            M.afrag = WT.afrag;
            M.kz = WT.kz;
            M.fsrc = fsrc;
            M.tags = tg;
            if (const char *v = sw_env(c, "HB_WMAC_WPE")) M.wpe = (u32)atoi(v);
            if (side) HB_CHECK(hipStreamWaitEvent(c->stream, c->ev_side1, 0), "hipStreamWaitEvent");
            HB_CHECK(hb_launch_wmac<NL>(M, c->stream), "hb_wmac_kernel launch");
            c->last_launches += M.nfull ? 1 : 0;
            const u64 with_data = (dlen + C - 1) / C < nb ? (dlen + C - 1) / C : nb;
            const u64 tail_end = cxx ? with_data : nb;
            if (tail_end > M.nfull) {
                EncodeArgs<NL> T = A;
                T.data = d + M.nfull * C;
                T.len = dlen - M.nfull * C;
                T.nblocks = tail_end - M.nfull;
                T.tags = tg + M.nfull * pi.tw;
                T.fv = fsrc + M.nfull * NL;
                HB_CHECK(hb_launch_mac<NL>(T, full16(pi, NL, C, T.data) ? 16 : 1, c->stream), "hb_mac_kernel launch");
                c->last_launches++;
            }
        }
        (void)d; (void)dlen; (void)nb; (void)tg; (void)fsrc; (void)align;
        return 0;
    };
    if (!small) {
        rc = wide_table();
        if (rc) return rc;
    }
    if (mf_layout) {
        // built on the host while the GPU runs the prefix kernel
        rc = mfma_tables(c, p, S, A.kz, mf_layout);
        if (rc) return rc;
        A.mfma = (u32)mf_layout;
        A.afrag = (const u32 *)c->afrag.p;
        mark("MFMA tables");
    }

    bool alpha_todo = small;   // the first small-input launch computes alpha too
    auto launch = [&](const uint8_t *d, u64 dlen, u64 nb, u64 base, uint8_t *tg) -> int {
        A.data = d;
        A.len = dlen;
        A.nblocks = nb;
        A.block_base = base;
        A.tags = tg;
        const int align = full16(pi, NL, C, d) ? 16 : 1;
        if (small) {
            // F(base + k): placed quad waves, queue slot 0 not cleared per
            // chunk (no job counter; tries and abandoned jobs add up); the
            // first launch also computes alpha_j R mod p beside them
            Prf2Args<NL> F2;
            memset(&F2, 0, sizeof F2);
            PrfArgs<NL> &F = F2.f;
            F.prf = A.prf;
            F.x0 = base;
            F.n = nb;
            F.out = (u32 *)c->vals.p;
            F.t0 = c->t0;
            F.queue = q0;
            const bool placed = use_quad(c, nb + S);
            if (alpha_todo) {
                int nra = 0;
                // hb_prf_pair_kernel gives F and alpha 16-job wave positions
                // of their own: ceil(nb/16) + ceil(S/16) of the grid's 16 G,
                // which can be one more than ceil((nb + S)/16) -- with the
                // grid capped at #CUs that last position does not exist
                // (e.g. nb = 65535, S = 1 on 256 CUs) and alpha would never
                // be computed.  Such a launch runs alpha on its own first.
                const u64 pair_pos = (nb + 15) / 16 + ((u64)S + 15) / 16;
                const bool pair_fits = pair_pos <= 16ull * (u64)quad_engine(c, nb + S).grid;
                if (!placed || !pair_fits || !make_prf<NL>(a_key, key_len, p_be, p_len, F2.pa, nra) || nra != nr) {
                    // (a different AES key length for alpha: its own launch first)
                    rc = run_prf<NL>(c, a_key, key_len, p_be, p_len, nullptr, 0, S, (u32 *)c->alpha_raw.p, 1, 0);
                    if (rc) return rc;
                    rc = run_mont<NL>(c, p, (const u32 *)c->alpha_raw.p, (u32 *)c->alpha_mont.p, S);
                    if (rc) return rc;
                    F2.S = 0;
                } else {
                    F2.S = S;
                }
                F2.mod = A.mod;
                const Limbs &r2 = r2_of(c, p, NL);
                for (int t = 0; t < NL; ++t) F2.r2[t] = r2[t];
                F2.amont = (u32 *)c->alpha_mont.p;
                F2.aqueue = q0 + HB_QSLOT;
                alpha_todo = false;
            }
            const EngineShape es = quad_engine(c, nb + F2.S);
            F.qchunk = es.chunk;
            F.place = placed ? 1u : 0u;
            if (!placed) {   // queue: one job per quad per refill, every CU
                HB_CHECK(hipMemsetAsync(q0, 0, sizeof(unsigned long long), c->stream), "hipMemsetAsync");
                HB_CHECK(hb_launch_prf<NL>(F, nr, 3, (int)c->num_cus, c->stream), "hb_prf_kernel launch");
            } else if (F2.S) {
                HB_CHECK(hb_launch_prf_pair<NL>(F2, nr, es.grid, c->stream), "hb_prf_pair_kernel launch");
            } else {
                HB_CHECK(hb_launch_prf<NL>(F, nr, 3, es.grid, c->stream), "hb_prf_kernel launch");
            }
            c->last_launches++;
            if (wide) {
                rc = wide_table();
                if (!rc) rc = wide_mac(d, dlen, nb, tg, (const u32 *)c->vals.p, align);
                return rc;
            }
            HB_CHECK(hb_launch_mac<NL>(A, align, c->stream), "hb_mac_kernel launch");
            c->last_launches++;
            return 0;
        }
        // queue[0] is the per-launch job counter (and queue[3] the retry
        // count); queue[1] accumulates tries
        HB_CHECK(hipMemsetAsync(q0, 0, sizeof(unsigned long long), c->stream), "hipMemsetAsync");
        if (!two_pass) {
            A.queue = q0;
            if (wide) A.fout = f_in_tags ? (u32 *)tg : (u32 *)c->vals.p;
            HB_CHECK(hb_launch_encode<NL>(A, nr, wide ? 0 : align, cxx ? 3 : 0, engine_grid(c, nb), c->stream),
                     "hb_encode_kernel launch");
            c->last_launches++;
            if (wide) return wide_mac(d, dlen, nb, tg, A.fout, align);
            return 0;
        }
        HB_CHECK(hipMemsetAsync(q0 + 3, 0, sizeof(unsigned long long), c->stream), "hipMemsetAsync");
        A.queue = q0;
        if (data_dev) HB_CHECK(hipEventRecord(c->ph[0], c->stream), "hipEventRecord");
        const int palign = wide ? 0 : align;
        if (wide) A.fout = f_in_tags ? (u32 *)tg : (u32 *)c->vals.p;
        HB_CHECK(hb_launch_encode<NL>(A, nr, palign, 1, engine_grid(c, nb), c->stream),
                 "hb_encode_first_kernel launch");
        if (data_dev) HB_CHECK(hipEventRecord(c->ph[1], c->stream), "hipEventRecord");
        HB_CHECK(hipMemsetAsync(q7, 0, sizeof(unsigned long long), c->stream), "hipMemsetAsync");
        A.queue = q7;
        HB_CHECK(hb_launch_encode<NL>(A, nr, palign, 2, engine_grid(c, A.retry_cap), c->stream),
                 "hb_encode_retry_kernel launch");
        if (data_dev) HB_CHECK(hipEventRecord(c->ph[2], c->stream), "hipEventRecord");
        c->ph_valid = data_dev;
        c->last_launches += 2;
        if (wide) return wide_mac(d, dlen, nb, tg, A.fout, align);
        return 0;
    };

    if (data_dev) {
        rc = launch(data, len, nblocks, block_base, dtags);
        if (rc) return rc;
        HB_CHECK(hipEventRecord(c->k1, c->stream), "hipEventRecord");
        if (flags & HB_ASYNC) {
            // kernels enqueued: hb_ctx_wait (or the next call) completes it
            c->pending = true;
            c->pend_q0 = q0;
            c->pend_q7 = q7;
            return 0;
        }
        HB_CHECK(hipEventSynchronize(c->k1), "encode");
        HB_CHECK(hipEventElapsedTime(&ms_total, c->k0, c->k1), "hipEventElapsedTime");
        mark("kernels");
    } else {
        // Host bytes: chunks of whole blocks double-buffered through the GPU,
        // H2D on the copy stream overlapping the encode kernels of the previous
        // chunk on the compute stream.
        HB_CHECK(c->data[0].ensure((size_t)(cb * C)), "hipMalloc(staging)");
        HB_CHECK(c->data[1].ensure((size_t)(cb * C)), "hipMalloc(staging)");
        std::unique_ptr<HostWindows> hw, tw;
        try {   // (a helper thread that cannot be started: copy unpinned)
            // (below 32 MiB the windows' helper threads and page-locking cost
            // more than the pageable copy they would speed up: a 1 MiB file
            // waited ~150 us for its first window, profiles/r05/w)
            const bool reg = (flags & HB_HOST_REGISTER) && len >= (32ull << 20);
            if (reg) hw.reset(new HostWindows(c, data, len, true));
            if (reg && !tags_dev)
                tw.reset(new HostWindows(c, tags, nblocks * pi.tw, false, (double)pi.tw / (double)C));
        } catch (const std::exception &) {
            hw.reset();
            tw.reset();
        }
        auto tags_back = [&](u64 k, u64 n, int buf) -> int {
            HB_CHECK(hipStreamWaitEvent(c->copy, c->done[buf], 0), "hipStreamWaitEvent");
            if (!tw) {
                HB_CHECK(hipMemcpyAsync(tags + k * pi.tw, dtags + k * pi.tw, (size_t)(n * pi.tw),
                                        hipMemcpyDeviceToHost, c->copy),
                         "hipMemcpyAsync(D2H tags)");
                return 0;
            }
            // pinned tag windows: one DMA per window piece
            HB_CHECK(tw->copy(dtags + k * pi.tw, (uintptr_t)(tags + k * pi.tw), (uintptr_t)(tags + (k + n) * pi.tw),
                              false),
                     "hipMemcpyAsync(D2H tags)");
            return 0;
        };
        u64 last_k0 = 0, last_nb = 0;
        for (u64 k0 = 0, it = 0; k0 < nblocks; k0 += cb, ++it) {
            const int b = (int)(it & 1);
            const u64 nb = nblocks - k0 < cb ? nblocks - k0 : cb;
            const u64 off = k0 * C;
            const u64 end = (k0 + nb) * C < len ? (k0 + nb) * C : len;
            const u64 bytes = end > off ? end - off : 0;
            if (it >= 2) HB_CHECK(hipStreamWaitEvent(c->copy, c->done[b], 0), "hipStreamWaitEvent");
            if (bytes && hw) {
                // pinned windows: one DMA per window piece of the chunk
                HB_CHECK(hw->copy(c->data[b].p, (uintptr_t)(data + off), (uintptr_t)(data + end), true),
                         "hipMemcpyAsync(H2D)");
            } else if (bytes) {
                HB_CHECK(hipMemcpyAsync(c->data[b].p, data + off, (size_t)bytes, hipMemcpyHostToDevice, c->copy),
                         "hipMemcpyAsync(H2D)");
            }
            HB_CHECK(hipEventRecord(c->copied[b], c->copy), "hipEventRecord");
            HB_CHECK(hipStreamWaitEvent(c->stream, c->copied[b], 0), "hipStreamWaitEvent");
            rc = launch((const uint8_t *)c->data[b].p, bytes, nb, block_base + k0, dtags + k0 * pi.tw);
            if (rc) return rc;
            HB_CHECK(hipEventRecord(c->done[b], c->stream), "hipEventRecord");
            // the previous chunk's tags go back on the copy stream behind this
            // chunk's H2D (which must not wait for the previous encode)
            if (it >= 1 && !tags_dev) rc = tags_back(k0 - cb, cb, 1 - b);
            if (rc) return rc;
            last_k0 = k0;
            last_nb = nb;
        }
        if (!tags_dev && nblocks) rc = tags_back(last_k0, last_nb, (int)(((nblocks - 1) / cb) & 1));
        if (rc) return rc;
        if (!tags_dev) {
            HB_CHECK(hipEventRecord(c->copied[0], c->copy), "hipEventRecord");
            HB_CHECK(hipStreamWaitEvent(c->stream, c->copied[0], 0), "hipStreamWaitEvent");
        }
        HB_CHECK(hipEventRecord(c->k1, c->stream), "hipEventRecord");
        HB_CHECK(hipEventSynchronize(c->k1), "encode");
        HB_CHECK(hipEventElapsedTime(&ms_total, c->k0, c->k1), "hipEventElapsedTime");
        if (hw) hw->finish();
        if (tw) tw->finish();
    }
    c->last_ms = ms_total;
    if (!tags_dev && data_dev)
        HB_CHECK(hipMemcpy(tags, dtags, (size_t)(nblocks * pi.tw), hipMemcpyDeviceToHost), "hipMemcpy(tags)");
    // every engine slot in one read: the encode's (0: first pass or the small
    // path's PRF, 7: retry pass) and any other launch's abandoned jobs
    unsigned long long qs[16 * HB_QSLOT];
    HB_CHECK(hipMemcpy(qs, c->queue, sizeof qs, hipMemcpyDeviceToHost), "hipMemcpy(queue)");
    const unsigned long long *q = qs, *r = qs + HB_QSLOT * HB_SLOT_RETRY;
    if (q[2] || r[2]) return fail(c, HB_EINVAL, "PRF rejection sampling did not terminate for some blocks");
    if (wide) {
        u32 st = 0;
        HB_CHECK(hipMemcpy(&st, WT.status, 4, hipMemcpyDeviceToHost), "hipMemcpy(status)");
        if (st) return fail(c, HB_EHIP, "internal: wide MAC digit table did not close");
    }
    if (tries_out) *tries_out = q[1] + r[1];
    for (int s = 0; s < 16; ++s)
        if (qs[s * HB_QSLOT + 2]) return fail(c, HB_EINVAL, "PRF rejection sampling did not terminate");
    return 0;
}

// ------------------------------------------------------------------ sums
// Column counters (ncols + 1) and the index flag word of hb_wsum_kernel,
// zero on allocation; the kernels leave them zero.
int ensure_ctl(hb_ctx *c, u32 ncols) {
    const size_t want = ((size_t)ncols + 2) * sizeof(unsigned int);
    if (c->ctl.n < want) {
        HB_CHECK(c->ctl.ensure(want < 4096 ? 4096 : want), "hipMalloc(ctl)");
        HB_CHECK(hipMemsetAsync(c->ctl.p, 0, c->ctl.n, c->stream), "hipMemsetAsync(ctl)");
    }
    return 0;
}

// The fused launches' limb sums: zero between operations (each closer
// re-zeroes what it used), so a grown buffer is zeroed whole.  Growth is
// told by the size, not the address: hipFree + hipMalloc may hand back the
// same address, and a pointer comparison then left the new tail holding stale
// memory (a wrong sigma after a prove with fewer columns on the context).
int ensure_facc(hb_ctx *c, size_t bytes) {
    const size_t had = c->facc.n;
    HB_CHECK(c->facc.ensure(bytes), "hipMalloc(facc)");
    if (c->facc.n != had) HB_CHECK(hipMemsetAsync(c->facc.p, 0, c->facc.n, c->stream), "hipMemsetAsync(facc)");
    return 0;
}

unsigned int *flags_word(hb_ctx *c) { return (unsigned int *)c->ctl.p + (c->ctl.n / sizeof(unsigned int) - 1); }

int ensure_hres(hb_ctx *c, size_t words) {
    if (c->hres_n >= words) return 0;
    if (c->hres) (void)hipHostFree(c->hres);
    c->hres = nullptr;
    c->hres_n = 0;
    // coherent: a fused prove's host polls the completion token while the
    // kernel still runs (finish_sums)
    HB_CHECK(hipHostMalloc((void **)&c->hres, words * 4, hipHostMallocCoherent), "hipHostMalloc");
    c->hres_n = words;
    return 0;
}

u32 wsum_grid(u64 nterms) {
    // one term per thread while the challenge is small (latency-bound
    // gathers), at most HB_WSUM_WG workgroups per column (the last one sums
    // the partials one per thread)
    // (measured at 10,000 terms: 4 / 16 / 40 terms per thread take 1.2x /
    // 2.7x / 7x as long -- the gathers of one thread do not overlap)
    u64 g = (nterms + HB_WSUM_WG - 1) / HB_WSUM_WG;
    if (g > HB_WSUM_WG) g = HB_WSUM_WG;
    return (u32)(g ? g : 1);
}

// Launch a weighted-sum pass with results in c->sums (ncols * NL + status).
// Completion tokens of hb_wsum_kernel launches: consecutive within an
// operation (an `accumulate` launch checks for its predecessor's, token - 1),
// never 0; restarted well before the counter would wrap.
u32 next_token(hb_ctx *c, bool first_of_operation) {
    if (first_of_operation && c->wsum_token > 0xfff00000u) c->wsum_token = 0;
    return ++c->wsum_token;
}

template <int NL>
int launch_wsum(hb_ctx *c, WsumArgs<NL> &A, int align) {
    const u32 gx = wsum_grid(A.nterms);
    HB_CHECK(c->partials.ensure((size_t)A.ncols * gx * NL * 4), "hipMalloc(partials)");
    HB_CHECK(c->sums.ensure(((size_t)A.ncols * NL + 2) * 4), "hipMalloc(sums)");
    if (int rc = ensure_ctl(c, A.ncols)) return rc;
    if (c->ctl_dirty) {
        // an earlier weighted sum did not complete (finish_sums): its column
        // counters may be left non-zero (hb_wsum_kernel, invariant I1)
        HB_CHECK(hipMemsetAsync(c->ctl.p, 0, c->ctl.n, c->stream), "hipMemsetAsync(ctl)");
        c->ctl_dirty = false;
    }
    A.partials = (u32 *)c->partials.p;
    A.ctl = (unsigned int *)c->ctl.p;
    A.flags = flags_word(c);
    // The finishers write the results (ncols values, status, token) straight
    // into the pinned host buffer the caller's values are read from: no D2H
    // copy (a blit launch and its latency, ~10 us of a ~0.22 ms prove) after
    // the sum.  $HB_SUMS_ON_DEVICE (test switch, A/B): device buffer + copy.
    const size_t words = (size_t)A.ncols * NL + 2;
    c->sums_in_hres = !sw_env(c, "HB_SUMS_ON_DEVICE");
    c->sums_polled = false;
    if (c->sums_in_hres) {
        if (int rc = ensure_hres(c, words)) return rc;
        A.out = c->hres;
        // the token word finish_sums checks: a freshly grown pinned buffer
        // (or an earlier operation) may hold any value there, this launch's
        // token included.  Cleared before the operation's first launch only:
        // an `accumulate` launch reads its predecessor's token from it.
        if (!A.accumulate) c->hres[words - 1] = 0;
    } else {
        A.out = (u32 *)c->sums.p;
        if (!A.accumulate) HB_CHECK(hipMemsetAsync(A.out + words - 1, 0, 4, c->stream), "hipMemsetAsync(token)");
    }
    A.token = next_token(c, !A.accumulate);
    HB_CHECK(hb_launch_wsum<NL>(A, align, (int)gx, c->stream), "hb_wsum_kernel launch");
    return 0;
}

// After the finalizing wsum: copy the results back (one D2H), check the
// completion token and the status word, write the ncols values big-endian
// (tw bytes each) to out.
template <int NL>
int finish_sums(hb_ctx *c, u32 ncols, u32 tw, uint8_t *out, bool cxx_index_check) {
    const size_t words = (size_t)ncols * NL + 2;
    if (!c->sums_in_hres) {
        if (int rc = ensure_hres(c, words)) return rc;
        HB_CHECK(hipMemcpyAsync(c->hres, c->sums.p, words * 4, hipMemcpyDeviceToHost, c->stream), "hipMemcpy");
    }
    if (c->sums_polled && !sw_env(c, "HB_SYNC_WAIT")) {
        // A fused prove writes its sums, status word and (after a system-scope
        // release) the completion token into the coherent pinned buffer from
        // the kernel's last wave: watch the token word itself instead of
        // waiting for the stream -- no completion signal and thread wake-up
        // on the prove's critical path.  Bounded by the stream: once it has
        // drained (or failed), a missing token is the mismatch below.
        // ($HB_SYNC_WAIT, test switch: hipStreamSynchronize as before.)
        const volatile u32 *tok = c->hres + (size_t)ncols * NL + 1;
        for (u32 spins = 1; *tok != c->wsum_token; ++spins) {
            if ((spins & 255u) == 0) {
                const hipError_t q = hipStreamQuery(c->stream);
                if (q == hipSuccess) break;
                if (q != hipErrorNotReady) HB_CHECK(q, "prove");
            }
            __builtin_ia32_pause();
        }
        std::atomic_thread_fence(std::memory_order_acquire);
    } else {
        // (a polled wait -- hipEventQuery in a loop -- measured slower than
        // this blocking one: 0.2118 vs 0.2041 ms per configs[4] proof,
        // profiles/r05/j)
        HB_CHECK(hipStreamSynchronize(c->stream), "prove");
    }
    if (c->hres[(size_t)ncols * NL + 1] != c->wsum_token) {
        // some column's finisher (or a batch) did not run: out[] is not this
        // operation's result (hb_wsum_kernel, I1).  Loud, and the counters are
        // cleared before the next weighted sum.
        c->ctl_dirty = true;
        return fail(c, HB_EHIP, "internal: weighted sum did not complete (completion token mismatch)");
    }
    const u32 st = c->hres[(size_t)ncols * NL];
    if (st & 2u) return fail(c, HB_EINVAL, "PRF rejection sampling did not terminate");
    if (st & 4u) {   // a fused launch's bounded wait ran out (hb_fused_close): its counters are suspect
        c->ctl_dirty = true;
        return fail(c, HB_EHIP, "internal: fused weighted sum timed out");
    }
    if ((st & 1u) && cxx_index_check)
        return fail(c, HB_EINVAL, "vector::_M_range_check: challenge index out of range");
    for (u32 k = 0; k < ncols; ++k) to_be(&c->hres[(size_t)k * NL], NL, out + (size_t)k * tw, tw);
    return 0;
}

int u64_be(u64 v, uint8_t out[8]) {
    for (int k = 0; k < 8; ++k) out[k] = (uint8_t)(v >> (56 - 8 * k));
    return 0;
}

// ------------------------------------------------------------------ prove
// Host-data gather: the sectors of challenged blocks as full ss-byte
// big-endian integers (a short last sector right-aligned, past EOF zero) --
// the reference's seek(pos) / read(ss) per sector (PySwizzle.py:353-355,
// cxx :763-765), offsets in unsigned int for the cxx prove.
struct Gather {
    const uint8_t *data;
    u64 len, C;
    u32 ss, S, tw;
    bool wrap32;
    const uint8_t *tags;
    // Indices [0, n) over `threads` host threads (contiguous slices): the
    // gather is random reads of a (mapped) file, bound by page-cache / DRAM
    // latency per block, so it scales with threads.
    void run_parallel(const u64 *idx, u64 n, uint8_t *blocks, uint8_t *gtags, int threads) const {
        // about 1,024 blocks per thread at least: a thread's start costs
        // ~20 us, the gather of a block well under 1 us
        u64 T = threads < 2 ? 1 : (u64)threads;
        if (T > n / 1024) T = n / 1024 ? n / 1024 : 1;
        if (T == 1) return run(idx, n, blocks, gtags);
        std::vector<std::thread> ts;
        for (u64 t = 0; t < T; ++t) {
            const u64 a = n * t / T, b = n * (t + 1) / T;
            ts.emplace_back([=] { run(idx + a, b - a, blocks + a * C, gtags + a * tw); });
        }
        for (auto &th : ts) th.join();
    }
    void run(const u64 *idx, u64 n, uint8_t *blocks, uint8_t *gtags) const {
        for (u64 i = 0; i < n; ++i) {
            const u64 ix = idx[i];
            uint8_t *dst = blocks + i * C;
            const u64 base = ix * C;
            if (!wrap32 && base + C <= len) {
                memcpy(dst, data + base, (size_t)C);
            } else {
                for (u32 j = 0; j < S; ++j) {
                    const u64 pos = wrap32 ? (u64)(u32)(base + (u64)j * ss) : base + (u64)j * ss;
                    const u64 r = pos >= len ? 0 : (len - pos < ss ? len - pos : ss);
                    memset(dst + (size_t)j * ss, 0, (size_t)(ss - r));
                    if (r) memcpy(dst + (size_t)j * ss + (ss - r), data + pos, (size_t)r);
                }
            }
            memcpy(gtags + i * tw, tags + ix * tw, tw);
        }
    }
};

// Host threads for the host-file prove gather: $HB_GATHER_THREADS, else
// the process's CPU share ($OMP_NUM_THREADS, as GPU boxes export it) capped
// at 16.
int gather_threads() {
    const char *e = getenv("HB_GATHER_THREADS");
    if (!e || !*e) e = getenv("OMP_NUM_THREADS");
    int t = e && *e ? atoi(e) : (int)std::thread::hardware_concurrency();
    if (t < 1) t = 1;
    return t > 16 ? 16 : t;
}

template <int NL>
int prove_impl(hb_ctx *c, const uint8_t *p_be, size_t p_len, const PrimeInfo &pi, u32 S,
               const uint8_t *chal_key, size_t key_len, u64 chunk_begin, u64 chunk_end, u64 chunks,
               const uint8_t *vmax_be, size_t vmax_len, const uint8_t *tags, u64 ntags,
               const uint8_t *data, u64 len, u32 flags, uint8_t *mu_out, uint8_t *sigma_out) {
    Limbs p = from_be(p_be, p_len, NL);
    const u64 C = (u64)pi.ss * S;
    const u32 ncols = S + 1;
    // cxx prove (shacham_waters_private.cxx:731-789): a challenge of at least
    // #tags chunks checks every block in order without the index PRF
    // (check_all, :754-755, 762); both PRFs are the cxx prf; sector offsets
    // are computed in unsigned int (:738, 762-763).
    const bool cxx = flags & HB_PRF_CXX;
    const bool check_all = cxx && chunks >= ntags;
    if (check_all) chunks = ntags;
    if (cxx && (ntags >> 32)) return fail(c, HB_EUNSUPPORTED, "cxx prove: more than 2^32 - 1 tags");
    if (chunk_end > chunks) chunk_end = chunks;
    if (chunk_begin > chunk_end) chunk_begin = chunk_end;
    const u64 n = chunk_end - chunk_begin;
    if (n == 0) {
        memset(mu_out, 0, (size_t)S * pi.tw);
        memset(sigma_out, 0, pi.tw);
        return 0;
    }
    if (c->prove_dirty) {
        // an earlier prove failed between its two launches: its counters
        // (normally zeroed by the finalizing workgroup) are cleared here
        HB_CHECK(hipMemsetAsync(c->queue + HB_QSLOT * 2, 0, 2 * HB_QSLOT * sizeof(unsigned long long), c->stream),
                 "hipMemsetAsync");
        if (c->ctl.n) HB_CHECK(hipMemsetAsync(c->ctl.p, 0, c->ctl.n, c->stream), "hipMemsetAsync");
        if (c->facc.n) HB_CHECK(hipMemsetAsync(c->facc.p, 0, c->facc.n, c->stream), "hipMemsetAsync");
        c->prove_dirty = false;
        c->ctl_dirty = false;
    }
    // stage 1: idx_i = KeyedPRF(key, ntags)(i), v_i = KeyedPRF(key, v_max)(i)   (PySwizzle.py:344-345)
    ProveArgs<NL> PA;
    memset(&PA, 0, sizeof PA);
    uint8_t nbe[8];
    u64_be(ntags, nbe);
    int nr = 0, nr2 = 0;
    if (!make_prf<2>(chal_key, key_len, nbe, 8, PA.pi, nr2) || !make_prf<NL>(chal_key, key_len, vmax_be, vmax_len, PA.pv, nr))
        return fail(c, HB_EINVAL, "invalid challenge key");
    make_mod<NL>(p, PA.mod);
    const Limbs &r2 = r2_of(c, p, NL);
    for (int t = 0; t < NL; ++t) PA.r2[t] = r2[t];
    HB_CHECK(c->idx.ensure((size_t)n * 8), "hipMalloc(idx)");
    HB_CHECK(c->wts.ensure((size_t)n * NL * 4), "hipMalloc(v)");
    if (int rc = ensure_ctl(c, ncols)) return rc;
    PA.i0 = chunk_begin;
    PA.n = n;
    PA.ntags = ntags;
    PA.check_all = check_all ? 1u : 0u;
    PA.idx = (u64 *)c->idx.p;
    PA.vm = (u32 *)c->wts.p;
    PA.t0 = c->t0;
    PA.queue = c->queue + HB_QSLOT * 2;   // slots 2 (index) and 3 (v), zero between operations
    PA.flags = flags_word(c);
    const int vnb = (bitlen_be(vmax_be, vmax_len) + 7) / 8;
    const int mode_i = cxx ? 2 : 0, mode_v = cxx ? (vnb % 16 ? 2 : 1) : 0;
    c->last_launches = 0;
    // (no timing events: hb_last_kernel_ms reports encodes, and a prove is
    // latency-bound -- every host API call is on its critical path)
    c->prove_dirty = true;
    const bool quad = !cxx && use_quad(c, 2 * n);
    const EngineShape es = quad ? quad_engine(c, 2 * n) : small_engine(c, 2 * n);
    PA.qchunk = es.chunk;
    bool data_dev = flags & HB_DATA_ON_DEVICE;
    bool tags_dev = flags & HB_TAGS_ON_DEVICE;
    // A host file that is small next to what the host gather would move (at
    // most twice its bytes, or 8 MiB) and fits a 4 GiB staging buffer goes
    // to the device whole -- one sequential H2D -- and is proved
    // device-resident (the fused launch where it applies), instead of a D2H
    // of the indices, a host gather of n random blocks and an H2D between
    // two launches.  $HB_NO_PROVE_UPLOAD and $HB_TEST_PROVE_BATCH (test
    // switches): the host gather.
    const u64 up_max = 2 * n * C > (8ull << 20) ? 2 * n * C : (8ull << 20);
    if (!data_dev && !cxx && !check_all && len <= up_max && len <= (4ull << 30) &&
        !sw_env(c, "HB_NO_PROVE_UPLOAD") && !sw_env(c, "HB_TEST_PROVE_BATCH")) {
        HB_CHECK(c->gup.ensure((size_t)(len ? len : 16)), "hipMalloc(file)");
        if (len) HB_CHECK(hipMemcpyAsync(c->gup.p, data, (size_t)len, hipMemcpyHostToDevice, c->stream), "H2D(file)");
        data = (const uint8_t *)c->gup.p;
        data_dev = true;
    }
    if (data_dev && !tags_dev) {
        // device-resident file, host tags: upload the tags (1/S of the file's
        // size at most) and gather on the device, instead of copying the
        // whole file back to the host
        HB_CHECK(c->tags.ensure((size_t)(ntags * pi.tw)), "hipMalloc(tags)");
        HB_CHECK(hipMemcpyAsync(c->tags.p, tags, (size_t)(ntags * pi.tw), hipMemcpyHostToDevice, c->stream),
                 "hipMemcpy(tags)");
        tags = (const uint8_t *)c->tags.p;
        tags_dev = true;
    }
    // Device-resident file and tags: the PRF kernel gathers each challenged
    // block and tag into a compact buffer as soon as its index is found
    // (hb_gather_block, under the still-running v chains), and the weighted
    // sum reads that buffer (mode 2) instead of n random blocks of the file.
    // PySwizzle mode (no check_all), up to 64 MiB of gathered bytes, and
    // layouts the gather copies in 16-byte pieces (file, tags, C and the tag
    // width 16-byte aligned: one lane copying a block byte by byte would
    // outlast the v chains); $HB_NO_PROVE_GATHER (test switch, A/B) keeps the
    // file-gathering sum.
    const u64 gstride = (n * C + 15) & ~15ull;
    const bool galign16 = (uintptr_t)data % 16 == 0 && (uintptr_t)tags % 16 == 0 && C % 16 == 0 && pi.tw % 16 == 0;
    const bool dev_gather = data_dev && tags_dev && !cxx && !check_all && galign16 &&
                            !sw_env(c, "HB_NO_PROVE_GATHER") && n * (C + pi.tw) <= (64ull << 20);
    // the index and v PRFs on disjoint halves of the grid (hb_prove_prf_kernel)
    const int pgrid = !check_all && es.grid < 2 ? 2 : es.grid;
    // quad engine: waves placed by SIMD, one v chain per SIMD where they fit
    // (hb_prove_place; needs at most 16 waves per workgroup for the jobs);
    // $HB_NO_PROVE_PLACE (test switch, A/B): waves race for the job queue
    const u64 pwaves = 2 * ((n + 15) / 16);
    PA.place = quad && pwaves <= 16ull * (u64)pgrid && !sw_env(c, "HB_NO_PROVE_PLACE") ? 1u : 0u;
    // Fused weighted sums (hb_prove_fused): placed quad waves, a device
    // gather, at most 48 jobs per workgroup whose blocks, tags and sums fit
    // the LDS arena, primes up to HB_FUSE_MAX_NL limbs (the summers' registers);
    // $HB_NO_PROVE_FUSE (test switch, A/B): the PRF launch + hb_wsum_kernel
    const u64 fcmax = (n + (u64)pgrid - 1) / (u64)pgrid;
    u32 fzoff[5];
    const bool fuse = dev_gather && PA.place && NL <= HB_FUSE_MAX_NL && ncols <= 256 && fcmax <= HB_FZ_MAXJOBS &&
                      hb_fz_layout((u32)fcmax, NL, ncols, C, pi.tw, fzoff) <= HB_FZ_BYTES &&
                      !sw_env(c, "HB_NO_PROVE_FUSE");
    if (fuse) {
        if (int rc = ensure_facc(c, (size_t)ncols * NL * 8)) return rc;
        if (c->ctl_dirty) {
            HB_CHECK(hipMemsetAsync(c->ctl.p, 0, c->ctl.n, c->stream), "hipMemsetAsync(ctl)");
            HB_CHECK(hipMemsetAsync(c->facc.p, 0, c->facc.n, c->stream), "hipMemsetAsync(facc)");
            c->ctl_dirty = false;
        }
        const size_t words = (size_t)ncols * NL + 2;
        if (int rc = ensure_hres(c, words)) return rc;
        // finish_sums polls this word for the new token: clear what an
        // earlier operation left there (a fused verify keeps mu in hres, and
        // the top limb of a small-topped prime's mu_{S-1} lands on this word)
        c->hres[(size_t)ncols * NL + 1] = 0;
        c->sums_in_hres = true;
        c->sums_polled = true;
        PA.fuse = 1u;
        PA.ncols = ncols;
        PA.fcmax = (u32)fcmax;
        PA.fsec16 = pi.ss == 4u * NL && pi.ss % 16 == 0 ? 1u : 0u;
        PA.ftag16 = pi.tw == 4u * NL ? 1u : 0u;
        PA.ftoken = next_token(c, true);
        PA.facc = (unsigned long long *)c->facc.p;
        PA.fctl = (unsigned int *)c->ctl.p;
        PA.fout = c->hres;
        PA.data = data;
        PA.len = len;
        PA.C = C;
        PA.ss = pi.ss;
        PA.S = S;
        PA.tw = pi.tw;
        PA.tags = tags;
        PA.galign16 = 1u;
    } else if (dev_gather) {
        HB_CHECK(c->gdev.ensure((size_t)(gstride + n * pi.tw)), "hipMalloc(gather)");
        PA.data = data;
        PA.len = len;
        PA.C = C;
        PA.ss = pi.ss;
        PA.S = S;
        PA.tw = pi.tw;
        PA.tags = tags;
        PA.gdata = (unsigned char *)c->gdev.p;
        PA.gtags = (unsigned char *)c->gdev.p + gstride;
        PA.galign16 = 1u;
    }
    HB_CHECK(hb_launch_prove_prf<NL>(PA, nr, quad ? 3 : mode_i, quad ? 3 : mode_v, pgrid, c->stream),
             "hb_prove_prf_kernel launch");
    c->last_launches++;

    // stage 2: mu_j = sum v_i m_{idx_i, j}, sigma = sum v_i tag[idx_i]   (PySwizzle.py:351-368)
    WsumArgs<NL> A;
    memset(&A, 0, sizeof A);
    make_mod<NL>(p, A.mod);
    A.ncols = ncols;
    A.C = C;
    A.ss = pi.ss;
    A.S = S;
    A.tw = pi.tw;
    A.wrap32 = cxx ? 1u : 0u;
    A.ntags = ntags;
    A.qslots = PA.queue;
    A.nslots = 2;
    int rc = 0;
    if (fuse) {
        // the sums were taken inside the PRF launch
    } else if (dev_gather) {
        A.mode = 2;
        A.w = (const u32 *)c->wts.p;
        A.nterms = n;
        A.data = PA.gdata;
        A.len = n * C;
        A.tags = PA.gtags;
        A.finalize = 1;
        rc = launch_wsum<NL>(c, A, full16(pi, NL, C, PA.gdata) ? 16 : 1);
        if (rc) return rc;
        c->last_launches++;
    } else if (data_dev && tags_dev) {
        A.mode = 0;
        A.idx = check_all ? nullptr : (const u64 *)c->idx.p;
        A.idx_base = chunk_begin;
        A.w = (const u32 *)c->wts.p;
        A.nterms = n;
        A.data = data;
        A.len = len;
        A.tags = tags;
        A.finalize = 1;
        rc = launch_wsum<NL>(c, A, full16(pi, NL, C, data) ? 16 : 1);
        if (rc) return rc;
        c->last_launches++;
    } else {
        // Host bytes: the challenged blocks are gathered on the host -- the
        // reference's seek/read per index -- in batches of <= 64 MiB staged
        // through the GPU; each batch adds onto the running sums.
        std::vector<u64> hidx((size_t)n);
        if (check_all) {
            for (u64 i = 0; i < n; ++i) hidx[(size_t)i] = chunk_begin + i;
        } else {
            HB_CHECK(hipMemcpyAsync(hidx.data(), c->idx.p, (size_t)n * 8, hipMemcpyDeviceToHost, c->stream),
                     "hipMemcpy(idx)");
        }
        HB_CHECK(hipStreamSynchronize(c->stream), "prove PRFs");
        std::vector<uint8_t> tagbuf;
        if (tags_dev) {   // rare: device tags with host data
            tagbuf.resize((size_t)(ntags * pi.tw));
            HB_CHECK(hipMemcpy(tagbuf.data(), tags, tagbuf.size(), hipMemcpyDeviceToHost), "hipMemcpy(tags)");
        }
        const uint8_t *htags = tags_dev ? tagbuf.data() : tags;
        // out-of-range indices (cxx prf after 81 tries) read as zero, reported at the end
        for (u64 i = 0; i < n; ++i)
            if (hidx[(size_t)i] >= ntags) hidx[(size_t)i] = 0;
        Gather G{data, len, C, pi.ss, S, pi.tw, cxx, htags};
        // batches of <= 64 MiB, gathered by host threads into pinned buffer
        // s = k % 2 while the GPU copies and sums batch k - 1 from the other
        // one (same stream: H2D(k) then wsum(k), in order)
        // 64 MiB batches: the two pinned buffers stay with the context (128 MiB
        // of page-locked host memory per context until hb_ctx_destroy)
        u64 per = (u64)((64ull << 20) / (C + pi.tw)) ? (64ull << 20) / (C + pi.tw) : 1;
        // test hook: smaller batches, to exercise the double buffering
        if (const char *t = sw_env(c, "HB_TEST_PROVE_BATCH")) {
            const u64 cap = (u64)strtoull(t, nullptr, 10);
            if (cap >= 1 && cap < per) per = cap;
        }
        const u64 bn = n < per ? n : per;
        const size_t stage = (size_t)(bn * C + bn * pi.tw);
        const int nbuf = n > bn ? 2 : 1;
        for (int s = 0; s < nbuf; ++s) {
            HB_CHECK(c->gstage[s].ensure(stage), "hipHostMalloc(staging)");
            HB_CHECK(c->data[s].ensure(stage), "hipMalloc(staging)");
        }
        const int threads = gather_threads();
        u64 k = 0;
        for (u64 b0 = 0; b0 < n; b0 += bn, ++k) {
            const u64 m = n - b0 < bn ? n - b0 : bn;
            const int s = (int)(k % 2);
            // batch k - 2's H2D from this pinned buffer must have completed
            if (k >= 2) HB_CHECK(hipEventSynchronize(c->copied[s]), "prove batch");
            uint8_t *hb = (uint8_t *)c->gstage[s].p;
            G.run_parallel(&hidx[(size_t)b0], m, hb, hb + bn * C, threads);
            uint8_t *db = (uint8_t *)c->data[s].p;
            HB_CHECK(hipMemcpyAsync(db, hb, (size_t)(m * C), hipMemcpyHostToDevice, c->stream), "H2D");
            HB_CHECK(hipMemcpyAsync(db + bn * C, hb + bn * C, (size_t)(m * pi.tw), hipMemcpyHostToDevice, c->stream),
                     "H2D");
            HB_CHECK(hipEventRecord(c->copied[s], c->stream), "hipEventRecord");
            A.mode = 2;
            A.w = (const u32 *)c->wts.p + b0 * NL;
            A.nterms = m;
            A.data = db;
            A.len = m * C;
            A.tags = db + bn * C;
            A.accumulate = b0 ? 1u : 0u;
            A.finalize = b0 + m == n ? 1u : 0u;
            rc = launch_wsum<NL>(c, A, full16(pi, NL, C, db) ? 16 : 1);
            if (rc) return rc;
            c->last_launches++;
        }
    }
    std::vector<uint8_t> out((size_t)ncols * pi.tw);
    rc = finish_sums<NL>(c, ncols, pi.tw, out.data(), cxx && !check_all);
    // the finalizing launch ran to its end (its status decides rc) unless the
    // completion token says otherwise: then its PRF slots were not cleared
    c->prove_dirty = c->ctl_dirty;
    // An uploaded host file above kGupKeep is not kept on the context (up to
    // 4 GiB of device memory otherwise held until hb_ctx_destroy, next to the
    // tags); its upload cost far more than the synchronize this needs.
    constexpr size_t kGupKeep = 256ull << 20;
    if (c->gup.n > kGupKeep) {
        (void)hipStreamSynchronize(c->stream);
        c->gup.release();
    }
    if (rc) return rc;
    memcpy(mu_out, out.data(), (size_t)S * pi.tw);
    memcpy(sigma_out, out.data() + (size_t)S * pi.tw, pi.tw);
    return 0;
}

// ------------------------------------------------------------------ verify
template <int NL>
int verify_impl(hb_ctx *c, const uint8_t *p_be, size_t p_len, const PrimeInfo &pi, u32 S,
                const uint8_t *f_key, const uint8_t *a_key, size_t key_len, u64 state_chunks,
                const uint8_t *chal_key, size_t chal_key_len, u64 chunks, const uint8_t *vmax_be,
                size_t vmax_len, const uint8_t *mu, uint8_t *rhs_out, bool cxx = false) {
    Limbs p = from_be(p_be, p_len, NL);
    // cxx verify (shacham_waters_private.cxx:791-842): cxx prf throughout,
    // check_all when the challenge covers every block (:822-827)
    const bool check_all = cxx && chunks >= state_chunks;
    if (check_all) chunks = state_chunks;
    c->last_launches = 0;
    if constexpr (NL <= HB_FUSE_MAX_NL) {
        // One launch (hb_verify_fused_kernel) when the quad engine takes the
        // challenge, every workgroup's share fits its LDS arena, alpha fits 16
        // jobs per workgroup and all four keys have the same AES round count;
        // $HB_NO_VERIFY_FUSE (test switch, A/B): the launch sequence below.
        const u64 jobs2 = 2 * chunks;
        if (!cxx && chunks && use_quad(c, jobs2) && !sw_env(c, "HB_NO_VERIFY_FUSE")) {
            const int G = quad_engine(c, jobs2).grid;
            const u64 fcmax = (chunks + (u64)G - 1) / (u64)G;
            u32 off[5];
            VerifyArgs<NL> V;
            memset(&V, 0, sizeof V);
            uint8_t nbe0[8];
            u64_be(state_chunks, nbe0);
            int n1 = 0, n2 = 0, n3 = 0, n4 = 0;
            if (fcmax <= HB_FZ_MAXJOBS && S <= 16ull * (u64)G &&
                hb_fz_layout((u32)fcmax, NL, 1, 4ull * NL, 8, off) <= HB_FZ_BYTES &&
                make_prf<2>(chal_key, chal_key_len, nbe0, 8, V.pi, n1) &&
                make_prf<NL>(chal_key, chal_key_len, vmax_be, vmax_len, V.pv, n2) &&
                make_prf<NL>(f_key, key_len, p_be, p_len, V.pf, n3) &&
                make_prf<NL>(a_key, key_len, p_be, p_len, V.pa, n4) && n1 == n2 && n2 == n3 && n3 == n4) {
                if (c->verify_dirty) {
                    HB_CHECK(hipMemsetAsync(c->queue + HB_QSLOT * 12, 0, 4 * HB_QSLOT * sizeof(unsigned long long),
                                            c->stream), "hipMemsetAsync");
                    if (c->ctl.n) HB_CHECK(hipMemsetAsync(c->ctl.p, 0, c->ctl.n, c->stream), "hipMemsetAsync");
                    if (c->facc.n) HB_CHECK(hipMemsetAsync(c->facc.p, 0, c->facc.n, c->stream), "hipMemsetAsync");
                    c->verify_dirty = false;
                    c->ctl_dirty = false;
                }
                if (int rc = ensure_ctl(c, 1)) return rc;
                if (int rc = ensure_facc(c, (size_t)NL * 8)) return rc;
                if (c->ctl_dirty) {
                    HB_CHECK(hipMemsetAsync(c->ctl.p, 0, c->ctl.n, c->stream), "hipMemsetAsync(ctl)");
                    HB_CHECK(hipMemsetAsync(c->facc.p, 0, c->facc.n, c->stream), "hipMemsetAsync(facc)");
                    c->ctl_dirty = false;
                }
                // results, status, token, then mu (read by the kernel from host memory)
                if (int rc = ensure_hres(c, (size_t)NL + 2 + (size_t)S * NL)) return rc;
                u32 *hmu = c->hres + NL + 2;
                for (u32 j = 0; j < S; ++j) {
                    Limbs m = from_be(mu + (size_t)j * pi.tw, pi.tw, NL);
                    memcpy(hmu + (size_t)j * NL, m.data(), NL * 4);
                }
                c->hres[NL + 1] = 0;   // the polled token word (tokens are never 0)
                make_mod<NL>(p, V.mod);
                const Limbs &r2 = r2_of(c, p, NL);
                for (int t = 0; t < NL; ++t) V.r2[t] = r2[t];
                V.i0 = 0;
                V.n = chunks;
                V.ntags = state_chunks;
                V.S = S;
                V.fcmax = (u32)fcmax;
                V.mu = hmu;
                V.t0 = c->t0;
                V.queue = c->queue + HB_QSLOT * 12;   // slots 12-15, zero between fused verifies
                V.flags = flags_word(c);
                V.qchunk = 16;
                V.facc = (unsigned long long *)c->facc.p;
                V.fctl = (unsigned int *)c->ctl.p;
                V.fout = c->hres;
                V.ftoken = next_token(c, true);
                c->sums_in_hres = true;
                c->sums_polled = true;
                c->last_launches = 1;
                c->verify_dirty = true;
                HB_CHECK(hb_launch_verify_fused<NL>(V, n1, G, c->stream), "hb_verify_fused_kernel launch");
                const int rc = finish_sums<NL>(c, 1, pi.tw, rhs_out, false);
                c->verify_dirty = c->ctl_dirty;
                return rc;
            }
        }
    }
    const int pmode = cxx ? (pi.tw % 16 ? 2 : 1) : 0;
    const int vmode = cxx ? ((bitlen_be(vmax_be, vmax_len) + 7) / 8 % 16 ? 2 : 1) : 0;
    const u64 nterms = chunks + S;
    uint8_t nbe[8];
    u64_be(state_chunks, nbe);
    HB_CHECK(c->idx.ensure((size_t)(chunks ? chunks : 1) * 8), "hipMalloc");
    HB_CHECK(c->vals.ensure((size_t)nterms * NL * 4), "hipMalloc");   // raw v_i | alpha_j
    HB_CHECK(c->wts.ensure((size_t)nterms * NL * 4), "hipMalloc");    // Montgomery weights
    HB_CHECK(c->vals2.ensure((size_t)nterms * NL * 4), "hipMalloc");  // F(idx_i) | mu_j
    u32 *raw = (u32 *)c->vals.p, *w = (u32 *)c->wts.p, *val = (u32 *)c->vals2.p;
    int rc = 0;
    if (chunks) {
        // index = KeyedPRF(key, state.chunks), v = KeyedPRF(key, v_max)   (PySwizzle.py:381-382)
        if (check_all) {
            std::vector<u64> iota(chunks);
            for (u64 i = 0; i < chunks; ++i) iota[i] = i;
            HB_CHECK(hipMemcpyAsync(c->idx.p, iota.data(), (size_t)chunks * 8, hipMemcpyHostToDevice, c->stream), "H2D");
            HB_CHECK(hipStreamSynchronize(c->stream), "H2D(idx)");
        } else {
            rc = run_prf<2>(c, chal_key, chal_key_len, nbe, 8, nullptr, 0, chunks, (u32 *)c->idx.p, 8, cxx ? 2 : 0);
            if (rc) return rc;
        }
        rc = run_prf<NL>(c, chal_key, chal_key_len, vmax_be, vmax_len, nullptr, 0, chunks, raw, 9, vmode);
        if (rc) return rc;
        // f.eval(index.eval(i))   (PySwizzle.py:389)
        rc = run_prf<NL>(c, f_key, key_len, p_be, p_len, (const u64 *)c->idx.p, 0, chunks, val, 10, pmode);
        if (rc) return rc;
    }
    // alpha.eval(j)   (PySwizzle.py:392)
    rc = run_prf<NL>(c, a_key, key_len, p_be, p_len, nullptr, 0, S, raw + chunks * NL, 11, pmode);
    if (rc) return rc;
    rc = run_mont<NL>(c, p, raw, w, nterms);
    if (rc) return rc;
    std::vector<u32> hmu((size_t)S * NL);
    for (u32 j = 0; j < S; ++j) {
        Limbs m = from_be(mu + (size_t)j * pi.tw, pi.tw, NL);
        memcpy(&hmu[(size_t)j * NL], m.data(), NL * 4);
    }
    HB_CHECK(hipMemcpyAsync(val + chunks * NL, hmu.data(), hmu.size() * 4, hipMemcpyHostToDevice, c->stream), "H2D");
    WsumArgs<NL> A;
    memset(&A, 0, sizeof A);
    make_mod<NL>(p, A.mod);
    A.mode = 1;
    A.ncols = 1;
    A.w = w;
    A.vals = val;
    A.nterms = nterms;
    A.S = S;
    A.finalize = 1;   // no PRF slots to collect (nslots = 0): checked below
    rc = launch_wsum<NL>(c, A, 1);
    if (rc) return rc;
    rc = finish_sums<NL>(c, 1, pi.tw, rhs_out, false);
    if (rc) return rc;
    return check_prf_slots(c);
}

}  // namespace

// ================================================================== C ABI
extern "C" {

int hb_abi_version(void) { return HB_ABI_VERSION; }

int hb_build_flags(void) {
#if defined(HB_EXPERIMENT_BUILD)
    int f = HB_BUILD_EXPERIMENT;
#else
    int f = 0;
#endif
    if (switch_gate()) f |= HB_BUILD_TEST_SWITCHES;
    return f;
}

uint32_t hb_test_switches(void) {
    if (!switch_gate()) return 0;
    u32 m = 0;
    for (const SwitchName &s : kSwitches) {
        const char *v = getenv(s.env);
        if (v && *v) m |= s.bit;
    }
    return m;
}

int hb_device_count(int *n) {
    if (!n) return HB_EINVAL;
    *n = 0;
    int d = 0;
    if (hipGetDeviceCount(&d) != hipSuccess) return HB_EHIP;
    *n = d;
    return 0;
}

int hb_device_pci_bus_id(int device, char *out, size_t n) {
    if (!out || n < 16) return HB_EINVAL;
    out[0] = 0;
    if (hipDeviceGetPCIBusId(out, (int)n, device) != hipSuccess) return HB_EHIP;
    return 0;
}

int hb_ctx_create(int device, hb_ctx **out) {
    if (!out) return HB_EINVAL;
    *out = nullptr;
    int ndev = 0;
    hipError_t e = hipGetDeviceCount(&ndev);
    if (e != hipSuccess || ndev == 0) {
        g_create_error = std::string("no usable HIP device: ") + (e != hipSuccess ? hipGetErrorString(e) : "0 devices");
        return HB_EHIP;
    }
    if (device < 0 || device >= ndev) {
        g_create_error = "device ordinal out of range";
        return HB_EINVAL;
    }
    hb_ctx *c = new hb_ctx();
    c->device = device;
    c->switches = switch_gate();   // the test-switch gate, read once per context
    auto bad = [&](hipError_t err, const char *what) {
        g_create_error = std::string(what) + ": " + hipGetErrorString(err);
        hb_ctx_destroy(c);
        return HB_EHIP;
    };
    if ((e = hipSetDevice(device)) != hipSuccess) return bad(e, "hipSetDevice");
    hipDeviceProp_t prop;
    if ((e = hipGetDeviceProperties(&prop, device)) != hipSuccess) return bad(e, "hipGetDeviceProperties");
    if (!strstr(prop.gcnArchName, "gfx950")) {
        g_create_error = std::string("libhbswizzle is built for gfx950 (MI355X); device is ") + prop.gcnArchName;
        hb_ctx_destroy(c);
        return HB_EUNSUPPORTED;
    }
    c->num_cus = prop.multiProcessorCount;
    if ((e = hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking)) != hipSuccess) return bad(e, "hipStreamCreate");
    c->own_stream = c->stream;
    if ((e = hipStreamCreateWithFlags(&c->copy, hipStreamNonBlocking)) != hipSuccess) return bad(e, "hipStreamCreate");
    if ((e = hipStreamCreateWithFlags(&c->side, hipStreamNonBlocking)) != hipSuccess) return bad(e, "hipStreamCreate");
    if ((e = hipEventCreateWithFlags(&c->ev_side0, hipEventDisableTiming)) != hipSuccess) return bad(e, "hipEventCreate");
    if ((e = hipEventCreateWithFlags(&c->ev_side1, hipEventDisableTiming)) != hipSuccess) return bad(e, "hipEventCreate");
    if ((e = hipEventCreate(&c->k0)) != hipSuccess) return bad(e, "hipEventCreate");
    if ((e = hipEventCreate(&c->k1)) != hipSuccess) return bad(e, "hipEventCreate");
    for (int k = 0; k < 3; ++k)
        if ((e = hipEventCreate(&c->ph[k])) != hipSuccess) return bad(e, "hipEventCreate");
    for (int b = 0; b < 2; ++b) {
        if ((e = hipEventCreateWithFlags(&c->copied[b], hipEventDisableTiming)) != hipSuccess) return bad(e, "hipEventCreate");
        if ((e = hipEventCreateWithFlags(&c->done[b], hipEventDisableTiming)) != hipSuccess) return bad(e, "hipEventCreate");
    }
    if ((e = hipEventCreateWithFlags(&c->ev_alpha, hipEventDisableTiming)) != hipSuccess) return bad(e, "hipEventCreate");
    if ((e = hipEventCreateWithFlags(&c->ev_h2d, hipEventDisableTiming)) != hipSuccess) return bad(e, "hipEventCreate");
    if ((e = hipMalloc(&c->t0, 256 * sizeof(u32))) != hipSuccess) return bad(e, "hipMalloc");
    if ((e = hipMemcpy(c->t0, aes_tables().t0, 256 * sizeof(u32), hipMemcpyHostToDevice)) != hipSuccess)
        return bad(e, "hipMemcpy");
    if ((e = hipMalloc(&c->queue, 16 * HB_QSLOT * sizeof(unsigned long long))) != hipSuccess) return bad(e, "hipMalloc");
    if ((e = hipMemset(c->queue, 0, 16 * HB_QSLOT * sizeof(unsigned long long))) != hipSuccess) return bad(e, "hipMemset");
    // pinned staging for the encode's alpha / MFMA-table round trips (S <= 64
    // without regrowing), allocated here rather than inside the first encode
    if ((e = c->hscratch.ensure(64u << 10)) != hipSuccess) return bad(e, "hipHostMalloc");
    *out = c;
    return HB_OK;
}

void hb_ctx_destroy(hb_ctx *c) {
    if (!c) return;
    (void)hipSetDevice(c->device);
    settle(c);
    if (c->stream) (void)hipStreamSynchronize(c->stream);
    if (c->copy) (void)hipStreamSynchronize(c->copy);
    if (c->side) (void)hipStreamSynchronize(c->side);
    DevBuf *bufs[] = {&c->alpha_raw, &c->alpha_mont, &c->xs, &c->vals, &c->vals2, &c->wts, &c->idx,
                      &c->partials, &c->sums, &c->data[0], &c->data[1], &c->tags, &c->blen, &c->gtags,
                      &c->pfx, &c->retry, &c->ctl, &c->afrag, &c->mseeds, &c->moffs, &c->mdig, &c->gdev,
                      &c->facc, &c->gup, &c->wpw, &c->wtab};
    for (DevBuf *b : bufs) b->release();
    if (c->hres) (void)hipHostFree(c->hres);
    c->gstage[0].release();
    c->gstage[1].release();
    c->hscratch.release();
    if (c->t0) (void)hipFree(c->t0);
    if (c->queue) (void)hipFree(c->queue);
    if (c->k0) (void)hipEventDestroy(c->k0);
    if (c->k1) (void)hipEventDestroy(c->k1);
    for (int k = 0; k < 3; ++k)
        if (c->ph[k]) (void)hipEventDestroy(c->ph[k]);
    if (c->ev_alpha) (void)hipEventDestroy(c->ev_alpha);
    if (c->ev_h2d) (void)hipEventDestroy(c->ev_h2d);
    for (int b = 0; b < 2; ++b) {
        if (c->copied[b]) (void)hipEventDestroy(c->copied[b]);
        if (c->done[b]) (void)hipEventDestroy(c->done[b]);
    }
    if (c->own_stream) (void)hipStreamDestroy(c->own_stream);
    if (c->copy) (void)hipStreamDestroy(c->copy);
    if (c->side) (void)hipStreamDestroy(c->side);
    if (c->ev_side0) (void)hipEventDestroy(c->ev_side0);
    if (c->ev_side1) (void)hipEventDestroy(c->ev_side1);
    delete c;
}

int hb_last_kernel_phases(hb_ctx *c, double *ms, uint32_t n) {
    if (!c || (!ms && n)) return HB_EINVAL;
    settle(c);
    if (!c->ph_valid || n == 0) return 0;
    hipEvent_t ev[5] = {c->k0, c->ph[0], c->ph[1], c->ph[2], c->k1};
    HB_CHECK(hipEventSynchronize(c->k1), "hipEventSynchronize");
    uint32_t k = 0;
    for (; k < 4 && k < n; ++k) {
        float f = 0.f;
        HB_CHECK(hipEventElapsedTime(&f, ev[k], ev[k + 1]), "hipEventElapsedTime");
        ms[k] = f;
    }
    return (int)k;
}

int hb_ctx_num_cus(const hb_ctx *c, int *out) {
    if (!c || !out) return HB_EINVAL;
    *out = c->num_cus;
    return 0;
}

int hb_ctx_set_stream(hb_ctx *c, void *stream) {
    if (!c) return HB_EINVAL;
    settle(c);
    HB_CHECK(hipSetDevice(c->device), "hipSetDevice");
    // the previous stream's work (e.g. this context's own) is ordered before
    // anything enqueued on the new one
    HB_CHECK(hipStreamSynchronize(c->stream), "hipStreamSynchronize");
    c->stream = stream ? (hipStream_t)stream : c->own_stream;
    return 0;
}

int hb_ctx_prepare(hb_ctx *c, uint32_t prime_bits) {
    if (!c) return HB_EINVAL;
    HB_CHECK(hipSetDevice(c->device), "hipSetDevice");
    int nl = nl_for_bits((int)prime_bits);
    if (!nl) return fail(c, HB_EUNSUPPORTED, "primes above 2048 bits are not supported by this build");
    if (nl < 8) nl = 8;
    HbLoadOnly load_only;
    PrefixArgs PA;
    memset(&PA, 0, sizeof PA);
    (void)hb_launch_prefix(PA, 14, 0, c->stream);
    PrfArgs<2> P2;
    memset(&P2, 0, sizeof P2);
    (void)hb_launch_prf<2>(P2, 14, 0, 0, c->stream);
    switch (nl) {
    case 8: prepare_nl<8>(c); break;
    case 16: prepare_nl<16>(c); break;
    case 32: prepare_nl<32>(c); break;
#if !defined(HB_NO_NL64)
    case 64: prepare_nl<64>(c); break;
#endif
    default: return fail(c, HB_EUNSUPPORTED, "primes above 2048 bits are not supported by this build");
    }
    (void)hipGetLastError();
    return 0;
}

int hb_ctx_wait(hb_ctx *c, uint64_t *tries_out) {
    if (!c) return HB_EINVAL;
    HB_CHECK(hipSetDevice(c->device), "hipSetDevice");
    settle(c);
    const int rc = c->pend_rc;
    if (rc) c->err = c->pend_err;
    if (tries_out) *tries_out = c->pend_tries;
    c->pend_rc = 0;
    c->pend_tries = 0;
    return rc;
}

const char *hb_last_error(const hb_ctx *c) { return c ? c->err.c_str() : g_create_error.c_str(); }

size_t hb_width(const uint8_t *p_be, size_t p_len) { return (size_t)(bitlen_be(p_be, p_len) + 7) / 8; }

uint64_t hb_block_count(const uint8_t *p_be, size_t p_len, uint32_t sectors, uint64_t len) {
    u64 ss = (u64)bitlen_be(p_be, p_len) / 8;
    u64 C = ss * sectors;
    return C ? len / C + 1 : 0;
}

static int prf_eval_common(hb_ctx *c, const uint8_t *key, size_t key_len, const uint8_t *range_be,
                           size_t range_len, const uint64_t *xs, const uint8_t *digests, size_t n,
                           uint8_t *out) {
    if (!c) return HB_EINVAL;
    settle(c);
    if (int rc = check_key(c, key_len)) return rc;
    const int bits = bitlen_be(range_be, range_len);
    if (bits == 0) return fail(c, HB_EINVAL, "PRF range must be positive");
    const int nl = nl_for_bits(bits);
    if (!nl) return fail(c, HB_EUNSUPPORTED, "PRF ranges above 2048 bits are not supported by this build");
    if (n == 0) return 0;
    HB_CHECK(hipSetDevice(c->device), "hipSetDevice");
    const u64 *xd = nullptr;
    const u32 *dd = nullptr;
    if (digests) {
        // digests: n x 32 bytes (SHA-256 output order) -> big-endian words
        std::vector<u32> w(n * 8);
        for (size_t i = 0; i < n * 8; ++i)
            w[i] = (u32)digests[4 * i] << 24 | (u32)digests[4 * i + 1] << 16 | (u32)digests[4 * i + 2] << 8 |
                   digests[4 * i + 3];
        HB_CHECK(c->xs.ensure(n * 32), "hipMalloc");
        HB_CHECK(hipMemcpyAsync(c->xs.p, w.data(), n * 32, hipMemcpyHostToDevice, c->stream), "H2D");
        HB_CHECK(hipStreamSynchronize(c->stream), "H2D(digests)");
        dd = (const u32 *)c->xs.p;
    } else {
        HB_CHECK(c->xs.ensure(n * 8), "hipMalloc");
        HB_CHECK(hipMemcpyAsync(c->xs.p, xs, n * 8, hipMemcpyHostToDevice, c->stream), "H2D");
        xd = (const u64 *)c->xs.p;
    }
    HB_CHECK(c->vals.ensure(n * (size_t)nl * 4), "hipMalloc");
    u32 *vd = (u32 *)c->vals.p;
    int rc = 0;
    switch (nl) {
    case 2: rc = run_prf<2>(c, key, key_len, range_be, range_len, xd, 0, n, vd, 6, 0, dd); break;
    case 8: rc = run_prf<8>(c, key, key_len, range_be, range_len, xd, 0, n, vd, 6, 0, dd); break;
    case 16: rc = run_prf<16>(c, key, key_len, range_be, range_len, xd, 0, n, vd, 6, 0, dd); break;
    case 32: rc = run_prf<32>(c, key, key_len, range_be, range_len, xd, 0, n, vd, 6, 0, dd); break;
#if !defined(HB_NO_NL64)
    default: rc = run_prf<64>(c, key, key_len, range_be, range_len, xd, 0, n, vd, 6, 0, dd); break;
#else
    default: return fail(c, HB_EUNSUPPORTED, "ranges above 1024 bits: not in this build");
#endif
    }
    if (rc) return rc;
    std::vector<u32> h(n * (size_t)nl);
    HB_CHECK(hipMemcpyAsync(h.data(), c->vals.p, h.size() * 4, hipMemcpyDeviceToHost, c->stream), "D2H");
    HB_CHECK(hipStreamSynchronize(c->stream), "hb_prf_kernel");
    if (int rc2 = check_prf_slots(c)) return rc2;
    const size_t nb = (size_t)(bits + 7) / 8;
    for (size_t i = 0; i < n; ++i) to_be(&h[i * nl], (size_t)nl, out + i * nb, nb);
    return 0;
}

int hb_prf_eval(hb_ctx *c, const uint8_t *key, size_t key_len, const uint8_t *range_be,
                size_t range_len, const uint64_t *xs, size_t n, uint8_t *out) {
    return prf_eval_common(c, key, key_len, range_be, range_len, xs, nullptr, n, out);
}

int hb_prf_eval_digests(hb_ctx *c, const uint8_t *key, size_t key_len, const uint8_t *range_be,
                        size_t range_len, const uint8_t *digests, size_t n, uint8_t *out) {
    if (!digests && n) return fail(c, HB_EINVAL, "digests buffer is NULL");
    return prf_eval_common(c, key, key_len, range_be, range_len, nullptr, digests, n, out);
}

int hb_cxx_prf_eval(hb_ctx *c, const uint8_t *key, size_t key_len, const uint8_t *limit_be,
                    size_t limit_len, const uint32_t *xs, size_t n, uint8_t *out) {
    if (!c) return HB_EINVAL;
    settle(c);
    if (int rc = check_key(c, key_len)) return rc;
    const int bits = bitlen_be(limit_be, limit_len);
    if (bits == 0) return fail(c, HB_EINVAL, "PRF limit must be positive");
    const int nl = nl_for_bits(bits);
    const size_t nb = (size_t)(bits + 7) / 8;
    if (!nl) return fail(c, HB_EUNSUPPORTED, "PRF limits above 2048 bits are not supported by this build");
    const int mode = nb % 16 ? 2 : 1;   // byte-granular CFB-128 unless whole blocks per try
    if (n == 0) return 0;
    HB_CHECK(hipSetDevice(c->device), "hipSetDevice");
    std::vector<u64> x64(n);
    for (size_t i = 0; i < n; ++i) x64[i] = xs[i];
    const int nlv = nl < 8 ? 8 : nl;
    HB_CHECK(c->xs.ensure(n * 8), "hipMalloc");
    HB_CHECK(c->vals.ensure(n * (size_t)nlv * 4), "hipMalloc");
    HB_CHECK(hipMemcpyAsync(c->xs.p, x64.data(), n * 8, hipMemcpyHostToDevice, c->stream), "H2D");
    int rc = 0;
    switch (nlv) {
    case 8: rc = run_prf<8>(c, key, key_len, limit_be, limit_len, (const u64 *)c->xs.p, 0, n, (u32 *)c->vals.p, 6, mode); break;
    case 16: rc = run_prf<16>(c, key, key_len, limit_be, limit_len, (const u64 *)c->xs.p, 0, n, (u32 *)c->vals.p, 6, mode); break;
    case 32: rc = run_prf<32>(c, key, key_len, limit_be, limit_len, (const u64 *)c->xs.p, 0, n, (u32 *)c->vals.p, 6, mode); break;
#if !defined(HB_NO_NL64)
    default: rc = run_prf<64>(c, key, key_len, limit_be, limit_len, (const u64 *)c->xs.p, 0, n, (u32 *)c->vals.p, 6, mode); break;
#else
    default: return fail(c, HB_EUNSUPPORTED, "ranges above 1024 bits: not in this build");
#endif
    }
    if (rc) return rc;
    std::vector<u32> h(n * (size_t)nlv);
    HB_CHECK(hipMemcpyAsync(h.data(), c->vals.p, h.size() * 4, hipMemcpyDeviceToHost, c->stream), "D2H");
    HB_CHECK(hipStreamSynchronize(c->stream), "hb_prf_kernel");
    if (int rc2 = check_prf_slots(c)) return rc2;
    for (size_t i = 0; i < n; ++i) to_be(&h[i * nlv], (size_t)nlv, out + i * nb, nb);
    return 0;
}

int hb_encode(hb_ctx *c, const uint8_t *p_be, size_t p_len, uint32_t sectors,
              const uint8_t *f_key, const uint8_t *alpha_key, size_t key_len,
              uint64_t block_base, const uint8_t *data, uint64_t len,
              uint64_t nblocks, uint8_t *tags, uint32_t flags, uint64_t *tries_out) {
    if (!c) return HB_EINVAL;
    settle(c);
    PrimeInfo pi;
    if (int rc = parse_prime(c, p_be, p_len, pi)) return rc;
    if (int rc = check_key(c, key_len)) return rc;
    if (sectors == 0) return fail(c, HB_EINVAL, "sectors must be positive");
    if (!tags && nblocks) return fail(c, HB_EINVAL, "tags buffer is NULL");
    if (!data && len) return fail(c, HB_EINVAL, "data buffer is NULL");
    if (tries_out) *tries_out = 0;
    if ((flags & HB_ASYNC) && (flags & (HB_DATA_ON_DEVICE | HB_TAGS_ON_DEVICE)) != (HB_DATA_ON_DEVICE | HB_TAGS_ON_DEVICE))
        return fail(c, HB_EINVAL, "HB_ASYNC needs device-resident data and tags");
    if (nblocks == 0) return 0;
    HB_CHECK(hipSetDevice(c->device), "hipSetDevice");
    switch (pi.nl) {
    case 8: return encode_impl<8>(c, p_be, p_len, pi, sectors, f_key, alpha_key, key_len, block_base, data, len, nblocks, tags, flags, tries_out);
    case 16: return encode_impl<16>(c, p_be, p_len, pi, sectors, f_key, alpha_key, key_len, block_base, data, len, nblocks, tags, flags, tries_out);
    case 32: return encode_impl<32>(c, p_be, p_len, pi, sectors, f_key, alpha_key, key_len, block_base, data, len, nblocks, tags, flags, tries_out);
#if !defined(HB_NO_NL64)
    default: return encode_impl<64>(c, p_be, p_len, pi, sectors, f_key, alpha_key, key_len, block_base, data, len, nblocks, tags, flags, tries_out);
#else
    default: return fail(c, HB_EUNSUPPORTED, "primes above 1024 bits: not in this build");
#endif
    }
}

int hb_prove_range(hb_ctx *c, const uint8_t *p_be, size_t p_len, uint32_t sectors,
                   const uint8_t *chal_key, size_t key_len, uint64_t chunks,
                   uint64_t chunk_begin, uint64_t chunk_end,
                   const uint8_t *vmax_be, size_t vmax_len, const uint8_t *tags, uint64_t ntags,
                   const uint8_t *data, uint64_t len, uint32_t flags, uint8_t *mu_out, uint8_t *sigma_out) {
    if (!c) return HB_EINVAL;
    settle(c);
    PrimeInfo pi;
    if (int rc = parse_prime(c, p_be, p_len, pi)) return rc;
    if (int rc = check_key(c, key_len)) return rc;
    if (sectors == 0) return fail(c, HB_EINVAL, "sectors must be positive");
    if (ntags == 0) return fail(c, HB_EINVAL, "tag is empty");
    const int vbits = bitlen_be(vmax_be, vmax_len);
    if (vbits == 0) return fail(c, HB_EINVAL, "v_max must be positive");
    if (vbits > 32 * pi.nl) return fail(c, HB_EUNSUPPORTED, "v_max wider than the prime's limb count");
    HB_CHECK(hipSetDevice(c->device), "hipSetDevice");
    switch (pi.nl) {
    case 8: return prove_impl<8>(c, p_be, p_len, pi, sectors, chal_key, key_len, chunk_begin, chunk_end, chunks, vmax_be, vmax_len, tags, ntags, data, len, flags, mu_out, sigma_out);
    case 16: return prove_impl<16>(c, p_be, p_len, pi, sectors, chal_key, key_len, chunk_begin, chunk_end, chunks, vmax_be, vmax_len, tags, ntags, data, len, flags, mu_out, sigma_out);
    case 32: return prove_impl<32>(c, p_be, p_len, pi, sectors, chal_key, key_len, chunk_begin, chunk_end, chunks, vmax_be, vmax_len, tags, ntags, data, len, flags, mu_out, sigma_out);
#if !defined(HB_NO_NL64)
    default: return prove_impl<64>(c, p_be, p_len, pi, sectors, chal_key, key_len, chunk_begin, chunk_end, chunks, vmax_be, vmax_len, tags, ntags, data, len, flags, mu_out, sigma_out);
#else
    default: return fail(c, HB_EUNSUPPORTED, "primes above 1024 bits: not in this build");
#endif
    }
}

int hb_prove(hb_ctx *c, const uint8_t *p_be, size_t p_len, uint32_t sectors,
             const uint8_t *chal_key, size_t key_len, uint64_t chunks,
             const uint8_t *vmax_be, size_t vmax_len, const uint8_t *tags, uint64_t ntags,
             const uint8_t *data, uint64_t len, uint32_t flags, uint8_t *mu_out, uint8_t *sigma_out) {
    return hb_prove_range(c, p_be, p_len, sectors, chal_key, key_len, chunks, 0, UINT64_MAX, vmax_be, vmax_len,
                          tags, ntags, data, len, flags, mu_out, sigma_out);
}

static int verify_rhs(hb_ctx *c, const uint8_t *p_be, size_t p_len, uint32_t sectors,
                      const uint8_t *f_key, const uint8_t *alpha_key, size_t key_len,
                      uint64_t state_chunks, const uint8_t *chal_key, size_t chal_key_len, uint64_t chunks,
                      const uint8_t *vmax_be, size_t vmax_len, const uint8_t *mu, uint8_t *rhs_out, bool cxx);

int hb_verify_rhs(hb_ctx *c, const uint8_t *p_be, size_t p_len, uint32_t sectors,
                  const uint8_t *f_key, const uint8_t *alpha_key, size_t key_len,
                  uint64_t state_chunks, const uint8_t *chal_key, size_t chal_key_len, uint64_t chunks,
                  const uint8_t *vmax_be, size_t vmax_len, const uint8_t *mu, uint8_t *rhs_out) {
    return verify_rhs(c, p_be, p_len, sectors, f_key, alpha_key, key_len, state_chunks, chal_key,
                      chal_key_len, chunks, vmax_be, vmax_len, mu, rhs_out, false);
}

int hb_cxx_verify_rhs(hb_ctx *c, const uint8_t *p_be, size_t p_len, uint32_t sectors,
                      const uint8_t *f_key, const uint8_t *alpha_key, size_t key_len,
                      uint64_t state_chunks, const uint8_t *chal_key, size_t chal_key_len, uint64_t chunks,
                      const uint8_t *vmax_be, size_t vmax_len, const uint8_t *mu, uint8_t *rhs_out) {
    if (c && (state_chunks >> 32)) return fail(c, HB_EUNSUPPORTED, "cxx verify: more than 2^32 - 1 blocks");
    return verify_rhs(c, p_be, p_len, sectors, f_key, alpha_key, key_len, state_chunks, chal_key,
                      chal_key_len, chunks, vmax_be, vmax_len, mu, rhs_out, true);
}

}  // extern "C"

static int verify_rhs(hb_ctx *c, const uint8_t *p_be, size_t p_len, uint32_t sectors,
                      const uint8_t *f_key, const uint8_t *alpha_key, size_t key_len,
                      uint64_t state_chunks, const uint8_t *chal_key, size_t chal_key_len, uint64_t chunks,
                      const uint8_t *vmax_be, size_t vmax_len, const uint8_t *mu, uint8_t *rhs_out, bool cxx) {
    if (!c) return HB_EINVAL;
    settle(c);
    PrimeInfo pi;
    if (int rc = parse_prime(c, p_be, p_len, pi)) return rc;
    if (int rc = check_key(c, key_len)) return rc;
    if (int rc = check_key(c, chal_key_len)) return rc;
    if (sectors == 0) return fail(c, HB_EINVAL, "sectors must be positive");
    if (chunks && state_chunks == 0) return fail(c, HB_EINVAL, "state has no chunks");
    const int vbits = bitlen_be(vmax_be, vmax_len);
    if (chunks && vbits == 0) return fail(c, HB_EINVAL, "v_max must be positive");
    if (vbits > 32 * pi.nl) return fail(c, HB_EUNSUPPORTED, "v_max wider than the prime's limb count");
    HB_CHECK(hipSetDevice(c->device), "hipSetDevice");
    switch (pi.nl) {
    case 8: return verify_impl<8>(c, p_be, p_len, pi, sectors, f_key, alpha_key, key_len, state_chunks, chal_key, chal_key_len, chunks, vmax_be, vmax_len, mu, rhs_out, cxx);
    case 16: return verify_impl<16>(c, p_be, p_len, pi, sectors, f_key, alpha_key, key_len, state_chunks, chal_key, chal_key_len, chunks, vmax_be, vmax_len, mu, rhs_out, cxx);
    case 32: return verify_impl<32>(c, p_be, p_len, pi, sectors, f_key, alpha_key, key_len, state_chunks, chal_key, chal_key_len, chunks, vmax_be, vmax_len, mu, rhs_out, cxx);
#if !defined(HB_NO_NL64)
    default: return verify_impl<64>(c, p_be, p_len, pi, sectors, f_key, alpha_key, key_len, state_chunks, chal_key, chal_key_len, chunks, vmax_be, vmax_len, mu, rhs_out, cxx);
#else
    default: return fail(c, HB_EUNSUPPORTED, "primes above 1024 bits: not in this build");
#endif
    }
}

extern "C" {

int hb_aes_cfb8(const uint8_t *key, size_t key_len, const uint8_t *iv, const uint8_t *in,
                uint8_t *out, size_t n, int encrypt) {
    AesKey k;
    if (!aes_expand(key, key_len, k)) return HB_EINVAL;
    aes_cfb8(k, iv, in, out, n, encrypt != 0);
    return 0;
}

int hb_aes_cfb128(const uint8_t *key, size_t key_len, const uint8_t *iv, const uint8_t *in,
                  uint8_t *out, size_t n, int encrypt) {
    AesKey k;
    if (!aes_expand(key, key_len, k)) return HB_EINVAL;
    aes_cfb128(k, iv, in, out, n, encrypt != 0);
    return 0;
}

int hb_last_kernel_ms(hb_ctx *c, double *ms, uint32_t *launches) {
    if (!c) return HB_EINVAL;
    // a pending HB_ASYNC encode is the last one: complete it first (its status
    // stays for hb_ctx_wait); like every call on a context, not concurrently
    // with another call on the same context
    if (c->pending && hipSetDevice(c->device) == hipSuccess) settle(c);
    if (ms) *ms = c->last_ms;
    if (launches) *launches = c->last_launches;
    return 0;
}

// ------------------------------------------------------------------ Merkle chunks
int hb_merkle_offsets(hb_ctx *c, const uint8_t *seeds, size_t seed_len, uint64_t nseeds, uint64_t filesz,
                      uint64_t chunksz, uint64_t *offsets) {
    if (!c) return HB_EINVAL;
    settle(c);
    if (int rc = check_key(c, seed_len)) return rc;
    if (nseeds == 0) return 0;
    if (!seeds || !offsets) return fail(c, HB_EINVAL, "NULL buffer");
    // Merkle.py:497-502: a chunk no larger than the file; range filesz - chunksz + 1
    if (filesz < chunksz) chunksz = filesz;
    const u64 range = filesz - chunksz + 1;
    HB_CHECK(hipSetDevice(c->device), "hipSetDevice");
    MerkleArgs A;
    memset(&A, 0, sizeof A);
    A.seed_len = (u32)seed_len;
    A.n = nseeds;
    if (range == 0) return fail(c, HB_EUNSUPPORTED, "Merkle chunk range of 2^64");
    A.R[0] = (u32)range;
    A.R[1] = (u32)(range >> 32);
    int bits = 0;
    for (u64 r = range; r; r >>= 1) ++bits;
    A.nb = (u32)(bits + 7) / 8;
    A.topmask = (1u << (bits - 8 * ((int)A.nb - 1))) - 1u;
    // SHA-256("0"): eval(0) hashes str(0) (util.py:91)
    static const u32 dig0[8] = {0x5feceb66u, 0xffc86f38u, 0xd952786cu, 0x6d696c79u,
                                0xc2dbc239u, 0xdd4e91b4u, 0x6729d73au, 0x27fb57e9u};
    memcpy(A.dig0, dig0, sizeof dig0);
    HB_CHECK(c->mseeds.ensure((size_t)nseeds * seed_len), "hipMalloc");
    HB_CHECK(c->moffs.ensure((size_t)nseeds * 8), "hipMalloc");
    HB_CHECK(hipMemcpyAsync(c->mseeds.p, seeds, (size_t)nseeds * seed_len, hipMemcpyHostToDevice, c->stream), "H2D");
    A.seeds = (const unsigned char *)c->mseeds.p;
    A.offsets = (u64 *)c->moffs.p;
    if (int rc = ensure_ctl(c, 1)) return rc;
    A.flags = flags_word(c);
    A.t0 = c->t0;
    const int nr = seed_len == 16 ? 10 : seed_len == 24 ? 12 : 14;
    HB_CHECK(hipMemsetAsync(A.flags, 0, 4, c->stream), "hipMemsetAsync");
    HB_CHECK(hb_launch_merkle_offsets(A, nr, c->stream), "hb_merkle_offsets_kernel launch");
    u32 fl = 0;
    HB_CHECK(hipMemcpyAsync(offsets, c->moffs.p, (size_t)nseeds * 8, hipMemcpyDeviceToHost, c->stream), "D2H");
    HB_CHECK(hipMemcpyAsync(&fl, A.flags, 4, hipMemcpyDeviceToHost, c->stream), "D2H");
    HB_CHECK(hipMemsetAsync(A.flags, 0, 4, c->stream), "hipMemsetAsync");   // zero between operations
    HB_CHECK(hipStreamSynchronize(c->stream), "hb_merkle_offsets_kernel");
    if (fl & 2u) return fail(c, HB_EINVAL, "PRF rejection sampling did not terminate");
    return 0;
}

int hb_merkle_chunk_hmacs(hb_ctx *c, const uint8_t *seeds, size_t seed_len, uint64_t nseeds,
                          const uint8_t *data_dev, uint64_t len, const uint64_t *offsets, uint64_t chunk_len,
                          uint8_t *digests) {
    if (!c) return HB_EINVAL;
    settle(c);
    if (seed_len == 0 || seed_len > 64) return fail(c, HB_EINVAL, "HMAC keys of 1..64 bytes");
    if (nseeds == 0) return 0;
    if (!seeds || !offsets || !digests || (!data_dev && chunk_len)) return fail(c, HB_EINVAL, "NULL buffer");
    for (u64 i = 0; i < nseeds; ++i)
        if (offsets[i] > len || len - offsets[i] < chunk_len)
            return fail(c, HB_EINVAL, "chunk past the end of the data");
    HB_CHECK(hipSetDevice(c->device), "hipSetDevice");
    MerkleArgs A;
    memset(&A, 0, sizeof A);
    A.seed_len = (u32)seed_len;
    A.n = nseeds;
    HB_CHECK(c->mseeds.ensure((size_t)nseeds * seed_len), "hipMalloc");
    HB_CHECK(c->moffs.ensure((size_t)nseeds * 8), "hipMalloc");
    HB_CHECK(c->mdig.ensure((size_t)nseeds * 32), "hipMalloc");
    HB_CHECK(hipMemcpyAsync(c->mseeds.p, seeds, (size_t)nseeds * seed_len, hipMemcpyHostToDevice, c->stream), "H2D");
    HB_CHECK(hipMemcpyAsync(c->moffs.p, offsets, (size_t)nseeds * 8, hipMemcpyHostToDevice, c->stream), "H2D");
    A.seeds = (const unsigned char *)c->mseeds.p;
    A.hoff = (const u64 *)c->moffs.p;
    A.data = data_dev;
    A.len = len;
    A.chunksz = chunk_len;
    A.digests = (u32 *)c->mdig.p;
    HB_CHECK(hb_launch_hmac(A, c->stream), "hb_hmac_kernel launch");
    std::vector<u32> h((size_t)nseeds * 8);
    HB_CHECK(hipMemcpyAsync(h.data(), c->mdig.p, h.size() * 4, hipMemcpyDeviceToHost, c->stream), "D2H");
    HB_CHECK(hipStreamSynchronize(c->stream), "hb_hmac_kernel");
    for (size_t k = 0; k < h.size(); ++k)
        for (int b = 0; b < 4; ++b) digests[4 * k + b] = (uint8_t)(h[k] >> (24 - 8 * b));
    return 0;
}

int hb_fill_random(hb_ctx *c, uint8_t *dev_ptr, uint64_t len, uint64_t seed) {
    if (!c) return HB_EINVAL;
    settle(c);
    HB_CHECK(hipSetDevice(c->device), "hipSetDevice");
    HB_CHECK(hb_launch_fill(dev_ptr, len, seed, c->stream), "hb_fill_kernel launch");
    HB_CHECK(hipStreamSynchronize(c->stream), "hb_fill_kernel");
    return 0;
}

int hb_stream_read(hb_ctx *c, const void *dev_ptr, uint64_t len, double *ms) {
    if (!c || !dev_ptr) return HB_EINVAL;
    settle(c);
    HB_CHECK(hipSetDevice(c->device), "hipSetDevice");
    if ((uintptr_t)dev_ptr % 16) return fail(c, HB_EINVAL, "hb_stream_read needs a 16-byte aligned buffer");
    HB_CHECK(c->sums.ensure(64), "hipMalloc");
    HB_CHECK(hipEventRecord(c->k0, c->stream), "hipEventRecord");
    HB_CHECK(hb_launch_read(dev_ptr, len, (u32 *)c->sums.p, c->num_cus, c->stream), "hb_read_kernel launch");
    HB_CHECK(hipEventRecord(c->k1, c->stream), "hipEventRecord");
    HB_CHECK(hipEventSynchronize(c->k1), "hb_read_kernel");
    float t = 0.f;
    HB_CHECK(hipEventElapsedTime(&t, c->k0, c->k1), "hipEventElapsedTime");
    if (ms) *ms = t;
    return 0;
}

int hb_device_malloc(hb_ctx *c, uint64_t bytes, void **out) {
    if (!c || !out) return HB_EINVAL;
    HB_CHECK(hipSetDevice(c->device), "hipSetDevice");
    HB_CHECK(hipMalloc(out, bytes ? bytes : 1), "hipMalloc");
    return 0;
}

int hb_device_free(hb_ctx *c, void *p) {
    if (!c) return HB_EINVAL;
    settle(c);
    HB_CHECK(hipSetDevice(c->device), "hipSetDevice");
    HB_CHECK(hipFree(p), "hipFree");
    return 0;
}

int hb_host_register(hb_ctx *c, void *ptr, uint64_t bytes) {
    if (!c || !ptr || !bytes) return HB_EINVAL;
    HB_CHECK(hipSetDevice(c->device), "hipSetDevice");
    HB_CHECK(hipHostRegister(ptr, (size_t)bytes, hipHostRegisterDefault), "hipHostRegister");
    return 0;
}

int hb_host_unregister(hb_ctx *c, void *ptr) {
    if (!c || !ptr) return HB_EINVAL;
    HB_CHECK(hipSetDevice(c->device), "hipSetDevice");
    HB_CHECK(hipHostUnregister(ptr), "hipHostUnregister");
    return 0;
}

int hb_memcpy(hb_ctx *c, void *dst, const void *src, uint64_t bytes, int kind) {
    if (!c) return HB_EINVAL;
    settle(c);
    HB_CHECK(hipSetDevice(c->device), "hipSetDevice");
    hipMemcpyKind k = kind == 1 ? hipMemcpyHostToDevice : kind == 2 ? hipMemcpyDeviceToHost : hipMemcpyDeviceToDevice;
    HB_CHECK(hipMemcpy(dst, src, bytes, k), "hipMemcpy");
    return 0;
}

}  // extern "C"
