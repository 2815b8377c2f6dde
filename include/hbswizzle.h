/*
 * hbswizzle.h -- C ABI of libhbswizzle.so, the MI355X (gfx950) Swizzle
 * (Shacham-Waters private PDP) hot path.
 *
 * The reference has no C ABI: its native boundary is CPython/PyCXX
 * (cxx/Swizzle.hxx) and pure Python (heartbeat/PySwizzle/PySwizzle.py).  Each
 * entry point below names the reference interface whose work it replaces.
 * The Python mirror of the reference API (heartbeat_amd.PySwizzle) binds these
 * with ctypes; INTEGRATION.md shows the binding a maintainer would add.
 *
 * Conventions
 *   - Integers crossing the ABI (primes, ranges, tags, mu, sigma) are
 *     big-endian byte strings, like Crypto.Util.number.long_to_bytes.
 *   - Tag / proof values are fixed width: hb_width(p) = ceil(bitlen(p)/8)
 *     bytes each.
 *   - Buffers are caller-owned.  A pointer flagged *_ON_DEVICE is a device
 *     pointer on the context's GPU (e.g. a torch.cuda tensor's data_ptr());
 *     otherwise it is ordinary host memory.  Nothing allocated by the library
 *     is returned to the caller.
 *   - Return value 0 = success; negative = error, message in hb_last_error().
 *     The Python layer raises HeartbeatError(message) (heartbeat/exc.py:29-35).
 *   - One context per GPU; a context must not be used by two threads at once.
 *     Calls are synchronous (they return when results are in the caller's
 *     buffers).
 *   - There is no CPU fallback: every compute entry point runs HIP kernels and
 *     fails with an error if no GPU is usable.
 */
#ifndef HBSWIZZLE_H
#define HBSWIZZLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define HB_ABI_VERSION 1

/* flags */
#define HB_DATA_ON_DEVICE 1u   /* `data` is a device pointer */
#define HB_TAGS_ON_DEVICE 2u   /* `tags` / `tags_out` is a device pointer */
#define HB_ENCODE_SINGLE_PASS 4u  /* hb_encode: one-pass engine instead of the
                                     prefix-image first pass + retry pass (same
                                     tags; for A/B tests and measurements) */
#define HB_PRF_CXX 8u  /* hb_encode: the cxx Swizzle extension's PRF (cxx/prf.hxx:125-176:
                          CFB-128 over SHA256(LE32 i), <= 81 tries) and encode loop
                          (cxx/shacham_waters_private.cxx:638-702) instead of PySwizzle's
                          KeyedPRF; needs ByteCount(p) % 16 == 0 (the cxx API's 1024-bit
                          primes, 256-bit primes).  Tags differ from PySwizzle's.
                          Parity unpinned (Crypto++ absent). */

#define HB_ASYNC 16u  /* hb_encode with device-resident data and tags: return once the
                        encode kernels are enqueued on the context's stream (the
                        prologue -- alpha PRF, MFMA fragments -- still completes
                        first); hb_ctx_wait, or the context's next call, completes
                        it.  With hb_ctx_set_stream the kernels run on the
                        caller's stream ("an async variant takes a
                        hipStream_t"). */

#define HB_HOST_REGISTER 32u  /* hb_encode with host buffers: page-lock the file bytes
                                 read-only (hipHostRegisterReadOnly) and the host tag
                                 buffer for writing, in page-aligned windows of
                                 256 MiB pinned ahead of the copies by helper
                                 threads, and DMA the chunks straight from / into
                                 them (each window unpinned once its copies are
                                 done), instead of the runtime's pageable staging.
                                 For read-only mappings of files (the reference's
                                 file object, PySwizzle.py:299) and other large host
                                 buffers (files under 32 MiB are copied pageable:
                                 the windows would cost more than they save); a window that cannot be registered (e.g.
                                 already registered by the caller) is copied as is.
                                 Same tags. */

/* error codes */
#define HB_OK 0
#define HB_EINVAL -1
#define HB_EHIP -2
#define HB_ENOMEM -3
#define HB_EUNSUPPORTED -4

typedef struct hb_ctx hb_ctx;

int hb_abi_version(void);

/* Build properties.  HB_BUILD_EXPERIMENT: an A/B experiment build
 * (scripts/build_variant.sh) whose HB_EXP_* switches may emit wrong tags; the
 * Python package refuses such a library unless HB_LIB_PATH names it.
 * HB_BUILD_TEST_SWITCHES: HB_ENABLE_TEST_SWITCHES=1 is set in this process's
 * environment, so contexts created now honour the A/B and test switches
 * (hb_test_switches) -- never set for measurements. */
#define HB_BUILD_EXPERIMENT 1
#define HB_BUILD_TEST_SWITCHES 2
int hb_build_flags(void);

/* Provenance: hex SHA-256 of every source file of this library
 * (heartbeat_amd/csrc, this header) and of its compiler flags, as computed by
 * heartbeat_amd/build_id.py at build time; and those flags.  The Python
 * package refuses a library whose id does not match the tree it sits in. */
const char *hb_build_id(void);
const char *hb_build_flags_string(void);

/* The A/B and test switches (environment variables) a
 * context created now would honour, as a bit mask (HB_SW_*).  All of them
 * are ignored -- mask 0 -- unless HB_ENABLE_TEST_SWITCHES=1 is set when the
 * context is created; a context reads that gate once, at creation. */
#define HB_SW_NO_QUAD 1u
#define HB_SW_NO_MFMA 2u
#define HB_SW_MFMA_SECTOR_LOADS 4u
#define HB_SW_MFMA_LINE32 8u
#define HB_SW_MFMA_MIN_S 16u
#define HB_SW_NO_EARLY_LIST 32u
#define HB_SW_RETRY_CAP 64u
#define HB_SW_PROVE_BATCH 128u
#define HB_SW_TRACE_PHASES 256u
#define HB_SW_HOST_WINDOWS 512u   /* HB_HOST_WINDOW_MIB / HB_HOST_AHEAD: HB_HOST_REGISTER geometry */
#define HB_SW_NO_PROVE_GATHER 1024u  /* HB_NO_PROVE_GATHER: device proves sum straight from the file */
#define HB_SW_SUMS_ON_DEVICE 2048u   /* HB_SUMS_ON_DEVICE: weighted sums land in device memory + a D2H copy */
#define HB_SW_NO_PROVE_PLACE 4096u   /* HB_NO_PROVE_PLACE: prove PRF waves take jobs from the queue, not by SIMD */
#define HB_SW_NO_PROVE_FUSE 8192u    /* HB_NO_PROVE_FUSE: device proves sum in a second launch (hb_wsum_kernel) */
#define HB_SW_SYNC_WAIT 16384u       /* HB_SYNC_WAIT: a fused prove waits for its stream instead of polling its token */
#define HB_SW_NO_VERIFY_FUSE 32768u  /* HB_NO_VERIFY_FUSE: verify as a launch sequence (PRFs, mont, hb_wsum_kernel) */
#define HB_SW_NO_SMALL_ENCODE 65536u /* HB_NO_SMALL_ENCODE: the two-pass engine for small inputs too */
#define HB_SW_NO_PROVE_UPLOAD 131072u /* HB_NO_PROVE_UPLOAD: small host files are gathered on the host, not uploaded */
#define HB_SW_MID_BLOCKS 262144u     /* HB_MID_BLOCKS=n: up to n blocks per launch (default 17 x 256 x #CUs; 16 x for primes above 256 bits) take the queued quad-PRF + MAC path */
#define HB_SW_NO_WIDE 524288u       /* HB_NO_WIDE: primes above 256 bits keep the MAC inside the PRF kernels (VALU) instead of the split F-only passes + MFMA MAC (hb_wmac_kernel) */
#define HB_SW_WMAC_WPE 1048576u     /* HB_WMAC_WPE=1|3|5: hb_wmac_kernel built for another waves-per-SIMD bound (1: the compiler's choice) */
#define HB_SW_WIDE_SYNC_ALPHA 2097152u /* HB_WIDE_SYNC_ALPHA: the split encode computes alpha and its digit table on the compute stream, before the PRF passes, instead of beside them */
#define HB_SW_QCHUNK 4194304u       /* HB_QCHUNK=n: jobs per queue refill in the encode engines (default 256 up to 256-bit primes, 64 above; rounded up to a multiple of 64) */
uint32_t hb_test_switches(void);

/* Number of visible HIP devices (multi-GPU sharding of encode / prove opens
 * one context per device; contexts fail on non-gfx950 devices). */
int hb_device_count(int *n);

/* PCI bus id ("dddd:bb:dd.f", NUL-terminated, n >= 16) of HIP device
 * `device`: tells physically distinct GPUs apart (bench.py's
 * distinct_devices) whatever ordinal remapping a launcher applies. */
int hb_device_pci_bus_id(int device, char *out, size_t n);

/* Open a context on HIP device `device`.  Replaces nothing in the reference
 * (it runs on the host only); the reference's per-call state lives in
 * PySwizzle objects (PySwizzle.py:233-255). */
int hb_ctx_create(int device, hb_ctx **out);
void hb_ctx_destroy(hb_ctx *ctx);
/* Message of the last error on this context (or of the last failed
 * hb_ctx_create when ctx is NULL). */
const char *hb_last_error(const hb_ctx *ctx);

/* Compute units of the context's device (the small-input encode and the
 * prove size their launches by it; tests place inputs at those limits).
 * Replaces nothing in the reference. */
int hb_ctx_num_cus(const hb_ctx *ctx, int *out);

/* Enqueue this context's kernels on `stream` (a hipStream_t of the
 * context's device, e.g. torch.cuda.current_stream().cuda_stream), or on the
 * context's own stream again with NULL.  Waits for the work already enqueued
 * on the previous stream. */
int hb_ctx_set_stream(hb_ctx *ctx, void *stream);

/* Complete an HB_ASYNC hb_encode: wait for its kernels, check its PRF
 * counters.  Returns the status of the async encodes completed since the last
 * hb_ctx_wait -- the FIRST failure among them, 0 if none failed -- and
 * *tries_out (may be NULL) receives their PRF tries.  Read the tags after
 * this call. */
int hb_ctx_wait(hb_ctx *ctx, uint64_t *tries_out);

/* Load the GPU code of the kernels that encodes and proves with a prime of
 * `prime_bits` bits launch, ahead of the first such call (the HIP runtime
 * otherwise loads a kernel translation unit's code object inside its first
 * launch: ~5 ms for the 256-bit unit).  Optional; replaces nothing in the
 * reference (setup, like creating a library handle). */
int hb_ctx_prepare(hb_ctx *ctx, uint32_t prime_bits);

/* ceil(bitlen(p)/8): width of every tag / mu / sigma value. */
size_t hb_width(const uint8_t *p_be, size_t p_len);

/* Batched KeyedPRF.eval.
 * Replaces heartbeat/util.py:83-96 (KeyedPRF.eval) and, for the cxx twin's
 * callers, cxx/prf.hxx:125-145 (prf::evaluate) -- with PySwizzle semantics.
 * out[i] = KeyedPRF(key, range).eval(xs[i]), written big-endian with
 * ceil(bitlen(range)/8) bytes each.  key: 16, 24 or 32 bytes (AES-128/192/256).
 * xs and out are host buffers. */
int hb_prf_eval(hb_ctx *ctx, const uint8_t *key, size_t key_len,
                const uint8_t *range_be, size_t range_len,
                const uint64_t *xs, size_t n, uint8_t *out);

/* KeyedPRF.eval over caller-hashed inputs.
 * Replaces heartbeat/util.py:83-96 for inputs hb_prf_eval cannot take: the
 * reference hashes str(x) of ANY Python int (util.py:91), negative and wider
 * than 64 bits included.  digests: n x 32 bytes, digest i = SHA256(str(x_i));
 * out as hb_prf_eval. */
int hb_prf_eval_digests(hb_ctx *ctx, const uint8_t *key, size_t key_len,
                        const uint8_t *range_be, size_t range_len,
                        const uint8_t *digests, size_t n, uint8_t *out);

/* Merkle chunk positions.
 * Replaces the KeyedPRF call of heartbeat/Merkle/Merkle.py:497-504
 * (MerkleHelper.get_chunk_hash): with chunk = min(chunksz, filesz),
 *   offsets[i] = KeyedPRF(seed_i, filesz - chunk + 1).eval(0)
 * for nseeds seeds of seed_len (16, 24 or 32) bytes each (every seed is its
 * own AES key).  seeds and offsets are host buffers. */
int hb_merkle_offsets(hb_ctx *ctx, const uint8_t *seeds, size_t seed_len, uint64_t nseeds,
                      uint64_t filesz, uint64_t chunksz, uint64_t *offsets);

/* Merkle chunk leaves.
 * Replaces the HMAC loop of heartbeat/Merkle/Merkle.py:505-515:
 *   digests[i] = HMAC-SHA256(seed_i, data[offsets[i] : offsets[i] + chunk_len])
 * over a DEVICE-resident data buffer of len bytes (every chunk must lie
 * inside it); one GPU lane hashes one chunk (a serial SHA-256 stream).
 * seed_len: 1..64 bytes.  seeds, offsets (host) and digests (host,
 * nseeds * 32 bytes). */
int hb_merkle_chunk_hmacs(hb_ctx *ctx, const uint8_t *seeds, size_t seed_len, uint64_t nseeds,
                          const uint8_t *data_dev, uint64_t len, const uint64_t *offsets,
                          uint64_t chunk_len, uint8_t *digests);

/* Swizzle encode of a run of blocks.
 * Replaces heartbeat/PySwizzle/PySwizzle.py:296-309 (the encode loop) and
 * cxx/shacham_waters_private.cxx:672-697.  For k in [0, nblocks):
 *   tags[k] = (F(block_base + k) + sum_j alpha(j) * m_kj) mod p
 * with F = KeyedPRF(f_key, p), alpha = KeyedPRF(alpha_key, p), sector size
 * ss = bitlen(p)/8, block size C = sectors*ss and m_kj the big-endian integer
 * of data[k*C + j*ss : min(k*C + (j+1)*ss, len)] (0 when empty; sectors after
 * the first short one contribute 0, PySwizzle.py:304-306).
 * A whole-file PySwizzle.encode is block_base = 0, nblocks = len/C + 1
 * (hb_block_count); shards of a file pass their first block index as
 * block_base and only their own bytes.
 * tags: nblocks * hb_width(p) bytes.  *tries_out (may be NULL) receives the
 * total number of PRF tries spent on the F values (>= nblocks). */
int hb_encode(hb_ctx *ctx, const uint8_t *p_be, size_t p_len, uint32_t sectors,
              const uint8_t *f_key, const uint8_t *alpha_key, size_t key_len,
              uint64_t block_base, const uint8_t *data, uint64_t len,
              uint64_t nblocks, uint8_t *tags, uint32_t flags,
              uint64_t *tries_out);

/* The cxx prf, prf::evaluate(i) (cxx/prf.hxx:125-145), for n unsigned-int
 * inputs, keyed by key and bounded by limit (any limit up to 2048 bits; when
 * ByteCount(limit) is not a multiple of 16 the CFB-128 stream continues
 * mid-block across tries): out receives n values of ByteCount(limit)
 * big-endian bytes each. */
int hb_cxx_prf_eval(hb_ctx *ctx, const uint8_t *key, size_t key_len,
                    const uint8_t *limit_be, size_t limit_len,
                    const uint32_t *xs, size_t n, uint8_t *out);

/* len/C + 1: the number of tags PySwizzle.encode produces for a file. */
uint64_t hb_block_count(const uint8_t *p_be, size_t p_len, uint32_t sectors,
                        uint64_t len);

/* Swizzle prove.
 * Replaces heartbeat/PySwizzle/PySwizzle.py:333-370 and
 * cxx/shacham_waters_private.cxx:731-789:
 *   idx_i = KeyedPRF(chal_key, ntags)(i), v_i = KeyedPRF(chal_key, v_max)(i)
 *   mu_j  = sum_i v_i * m_{idx_i, j} mod p      (i < chunks)
 *   sigma = sum_i v_i * tags[idx_i]    mod p
 * tags: ntags * hb_width(p) bytes.  data: the whole file (len bytes).
 * mu_out: sectors * hb_width(p) bytes, sigma_out: hb_width(p) bytes (host).
 * With HB_PRF_CXX: the cxx extension's prove (shacham_waters_private.cxx:731-789)
 * -- idx_i and v_i from the cxx prf (cxx/prf.hxx), every block in order when
 * chunks >= ntags (check_all, :754-762), and block offsets computed as
 * (unsigned int)(idx * sectors * ss) like the reference (:738, 763; differs
 * from PySwizzle for blocks past 4 GiB).  Parity unpinned (Crypto++ absent). */
int hb_prove(hb_ctx *ctx, const uint8_t *p_be, size_t p_len, uint32_t sectors,
             const uint8_t *chal_key, size_t key_len, uint64_t chunks,
             const uint8_t *vmax_be, size_t vmax_len,
             const uint8_t *tags, uint64_t ntags,
             const uint8_t *data, uint64_t len, uint32_t flags,
             uint8_t *mu_out, uint8_t *sigma_out);

/* The part of hb_prove over challenge indices [chunk_begin, chunk_end) of a
 * `chunks`-index challenge: mu_out / sigma_out receive that range's sums mod p.
 * The sums of a partition of [0, chunks) add (mod p) to hb_prove's result:
 * a prove sharded over several GPUs (one context each) is one call per GPU
 * plus a host-side sum of S + 1 values mod p.  hb_prove is chunk_begin = 0,
 * chunk_end = UINT64_MAX.  Replaces the same loop as hb_prove
 * (PySwizzle.py:351-368; cxx shacham_waters_private.cxx:757-788). */
int hb_prove_range(hb_ctx *ctx, const uint8_t *p_be, size_t p_len, uint32_t sectors,
                   const uint8_t *chal_key, size_t key_len, uint64_t chunks,
                   uint64_t chunk_begin, uint64_t chunk_end,
                   const uint8_t *vmax_be, size_t vmax_len,
                   const uint8_t *tags, uint64_t ntags,
                   const uint8_t *data, uint64_t len, uint32_t flags,
                   uint8_t *mu_out, uint8_t *sigma_out);

/* Right-hand side of PySwizzle.verify (PySwizzle.py:381-394) for a decrypted
 * state:  rhs = sum_i v_i * F(idx_i) + sum_j alpha(j) * mu_j  mod p.
 * The caller compares rhs with proof.sigma.  mu: sectors * hb_width(p) bytes
 * (each value must be < 2^(8*width)). */
int hb_verify_rhs(hb_ctx *ctx, const uint8_t *p_be, size_t p_len, uint32_t sectors,
                  const uint8_t *f_key, const uint8_t *alpha_key, size_t key_len,
                  uint64_t state_chunks,
                  const uint8_t *chal_key, size_t chal_key_len, uint64_t chunks,
                  const uint8_t *vmax_be, size_t vmax_len,
                  const uint8_t *mu, uint8_t *rhs_out);

/* Right-hand side of the cxx extension's verify (shacham_waters_private.cxx:
 * 791-842) for a decrypted state: the same sum as hb_verify_rhs with the cxx
 * prf (cxx/prf.hxx) for index, v, f and alpha, and every block in order when
 * chunks >= state_chunks (check_all, :822-827).  Parity unpinned. */
int hb_cxx_verify_rhs(hb_ctx *ctx, const uint8_t *p_be, size_t p_len, uint32_t sectors,
                      const uint8_t *f_key, const uint8_t *alpha_key, size_t key_len,
                      uint64_t state_chunks,
                      const uint8_t *chal_key, size_t chal_key_len, uint64_t chunks,
                      const uint8_t *vmax_be, size_t vmax_len,
                      const uint8_t *mu, uint8_t *rhs_out);

/* Host AES-CFB8 (segment 8, any 16-byte IV) for PySwizzle State
 * encrypt/decrypt (PySwizzle.py:162-195): 64 bytes per call, not a hot path.
 * encrypt = 1 encrypts, 0 decrypts. */
int hb_aes_cfb8(const uint8_t *key, size_t key_len, const uint8_t *iv,
                const uint8_t *in, uint8_t *out, size_t n, int encrypt);

/* Host AES-CFB128 (full-block feedback, no padding) for the cxx extension's
 * State encrypt-and-sign (cxx/shacham_waters_private.cxx:169-306, Crypto++
 * CFB_Mode<AES>): a few dozen bytes per call, not a hot path. */
int hb_aes_cfb128(const uint8_t *key, size_t key_len, const uint8_t *iv,
                  const uint8_t *in, uint8_t *out, size_t n, int encrypt);

/* Device timing of the last hb_encode on this context: milliseconds spent in
 * the encode kernel (HIP events on the kernel's stream), and launch count.  A
 * pending HB_ASYNC encode is completed first (its status stays for
 * hb_ctx_wait). */
int hb_last_kernel_ms(hb_ctx *ctx, double *ms, uint32_t *launches);

/* Phase times of the last device-resident two-pass encode on this context
 * (ms[0..3]: the set-up kernels -- prefix image, MAC tables --, the first-try
 * pass, the retry pass, the split wide-prime MAC (0 when the MAC ran inside the
 * PRF passes)), from events between its launches.  Returns the number of
 * values written (at most n and 4; 0 when the last encode was not such a
 * launch), negative on error.  Replaces nothing in the reference
 * (instrumentation, like hb_last_kernel_ms). */
int hb_last_kernel_phases(hb_ctx *ctx, double *ms, uint32_t n);

/* Device memory helpers so that callers without a GPU framework (e.g. a cgo or
 * JNI binding) can hold a device-resident file: allocate, copy
 * (kind 1 = host->device, 2 = device->host, 3 = device->device), free. */
int hb_device_malloc(hb_ctx *ctx, uint64_t bytes, void **out);
int hb_device_free(hb_ctx *ctx, void *ptr);
int hb_memcpy(hb_ctx *ctx, void *dst, const void *src, uint64_t bytes, int kind);

/* Page-lock (pin) an existing host buffer for the device of ctx, e.g. the file
 * bytes and the tag buffer of a host-path hb_encode: pinned chunks are copied
 * by DMA at the full PCIe rate and overlap the encode of the previous chunk
 * (pageable ones go through a driver staging copy).  The reference reads the
 * file through Python read() calls (PySwizzle.py:299; cxx/PythonSeekableFile.hxx:47-54);
 * this is the native replacement's staging.  Unregister before freeing. */
int hb_host_register(hb_ctx *ctx, void *ptr, uint64_t bytes);
int hb_host_unregister(hb_ctx *ctx, void *ptr);

/* Fill len bytes of device memory with the synthetic SplitMix64 stream used by
 * the benchmarks and tests: byte k = byte (k mod 8) (little-endian) of
 * splitmix64(seed ^ (2*(k/16) + ((k mod 16) >= 8)) * 0xD1B54A32D192ED03). */
int hb_fill_random(hb_ctx *ctx, uint8_t *dev_ptr, uint64_t len, uint64_t seed);

/* Measurement helper (no reference counterpart): read len bytes of device
 * memory once with streaming 16-byte loads; *ms = kernel time.  bench.py
 * reports len / ms as the measured HBM read peak beside the vendor figure. */
int hb_stream_read(hb_ctx *ctx, const void *dev_ptr, uint64_t len, double *ms);

#ifdef __cplusplus
}
#endif
#endif /* HBSWIZZLE_H */
