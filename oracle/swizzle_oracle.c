/*
 * swizzle_oracle.c -- CPU restatement of the reference PySwizzle hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and the
 * cpu_baseline leg of bench.py may load this library, and only as the checker
 * (or as the timed CPU baseline).  The product (heartbeat_amd) never links or
 * calls it.
 *
 * Parity pinning: checked against golden vectors produced by the unmodified
 * reference PySwizzle (tests/golden/make_golden.py -> tests/golden/ JSON fixtures) in
 * tests/test_oracle.py.
 *
 * What it restates (file:line in /root/reference):
 *   hbo_prf_eval   heartbeat/util.py:83-96   KeyedPRF.eval: fresh AES-CFB8
 *                  (segment 8 bit, IV = 0^16) per eval over
 *                  pad(SHA256(decimal(x)), ceil(bitlen(R)/8)) (util.py:52-64),
 *                  masked to bitlen(R) bits (util.py:81), rejection sampled with
 *                  the CFB stream continuing across tries (util.py:89-96).
 *   hbo_encode     heartbeat/PySwizzle/PySwizzle.py:279-314
 *                  tag_i = (F(i) + sum_j alpha(j) * m_ij) mod p, sectors read
 *                  as right-aligned big-endian integers, stop at first short
 *                  read (:298-306).  Always floor(L/C)+1 tags.
 *   hbo_prove      PySwizzle.py:333-370
 *   hbo_verify     PySwizzle.py:372-395
 *   hbo_cxx_prf_eval / hbo_cxx_encode (mode 1): the cxx Swizzle extension's
 *                  PRF and encode loop, cxx/prf.hxx:97-176 (+ cxx/clz.h:36-48)
 *                  and cxx/shacham_waters_private.cxx:638-702: CFB-128 (full
 *                  block feedback, IV 0, resynchronised per evaluate) over
 *                  SHA256(LE32(i)) padded to ByteCount(limit), stream continuing
 *                  across tries, at most 81 tries; sigma %= p only after a
 *                  sector was read.  PARITY UNPINNED: Crypto++ is absent here,
 *                  so no reference output pins it; OpenSSL's
 *                  CFB-128 is the same primitive as CFB_Mode<AES> with full-block
 *                  feedback (SP 800-38A vectors).
 *
 * Arithmetic: OpenSSL BIGNUM (exact).  AES/SHA: OpenSSL EVP (AES-NI when the
 * host has it).  Threads: hbo_encode splits the block range into contiguous
 * slices over `nthreads` pthreads (used as the multi-core CPU baseline).
 */
#include <openssl/bn.h>
#include <openssl/evp.h>
#include <openssl/sha.h>
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#define HBO_MAX_NB 1024

typedef struct {
    EVP_CIPHER_CTX *ctx;
    int mode;               /* 0 KeyedPRF (util.py), 1 cxx prf (prf.hxx) */
    BIGNUM *range;
    int nb;                 /* ceil(bitlen(range)/8)          util.py:92 */
    unsigned char topmask;  /* mask on the most significant byte, util.py:81 */
} prf_t;

static const EVP_CIPHER *cfb8_for(size_t keylen) {
    switch (keylen) {
    case 16: return EVP_aes_128_cfb8();
    case 24: return EVP_aes_192_cfb8();
    case 32: return EVP_aes_256_cfb8();
    default: return NULL;
    }
}

static const EVP_CIPHER *cfb128_for(size_t keylen) {
    switch (keylen) {
    case 16: return EVP_aes_128_cfb128();
    case 24: return EVP_aes_192_cfb128();
    case 32: return EVP_aes_256_cfb128();
    default: return NULL;
    }
}

/* cxx/clz.h:36-48 (the build never defines HAVE_GNU_CLZ): leading zeros of a
 * positive int in 32 bits */
static unsigned cxx_clz(int x) {
    unsigned n = 0;
    if (x == 0) return 32;
    while (!(x & (int)0x80000000u)) { n++; x = (int)((unsigned)x << 1); }
    return n;
}

static int prf_init_mode(prf_t *f, const unsigned char *key, size_t keylen,
                         const unsigned char *range_be, size_t range_len, int mode);

static int prf_init(prf_t *f, const unsigned char *key, size_t keylen,
                    const unsigned char *range_be, size_t range_len) {
    return prf_init_mode(f, key, keylen, range_be, range_len, 0);
}

static int prf_init_mode(prf_t *f, const unsigned char *key, size_t keylen,
                         const unsigned char *range_be, size_t range_len, int mode) {
    static const unsigned char zero_iv[16] = {0};
    const EVP_CIPHER *c = mode ? cfb128_for(keylen) : cfb8_for(keylen);
    f->mode = mode;
    int bits;
    if (!c) return -1;
    f->range = BN_bin2bn(range_be, (int)range_len, NULL);
    bits = BN_num_bits(f->range);
    if (bits == 0) { BN_free(f->range); return -2; }   /* range 0: reference never terminates */
    f->nb = (bits + 7) / 8;
    if (f->nb > HBO_MAX_NB) { BN_free(f->range); return -3; }
    if (mode) {   /* set_limit, prf.hxx:97-116: ByteCount, mask from clz of the top byte */
        unsigned char top = range_be[range_len - (size_t)f->nb];
        unsigned char m = 0;
        int i;
        for (i = 0; i < (int)(32 - cxx_clz(top)); i++) m |= (unsigned char)(1u << i);
        f->topmask = m;
    } else {
        int topbits = bits - 8 * (f->nb - 1);
        f->topmask = (unsigned char)((1u << topbits) - 1u);
    }
    f->ctx = EVP_CIPHER_CTX_new();
    EVP_EncryptInit_ex(f->ctx, c, NULL, key, zero_iv);
    return 0;
}

static void prf_free(prf_t *f) {
    EVP_CIPHER_CTX_free(f->ctx);
    BN_free(f->range);
}

/* KeyedPRF.eval of the message str(x) (dec, n bytes) -> out (BIGNUM);
 * returns number of tries. */
static int prf_eval_msg(prf_t *f, const char *dec, size_t n, BIGNUM *out) {
    static const unsigned char zero_iv[16] = {0};
    unsigned char digest[32], data[HBO_MAX_NB], ct[HBO_MAX_NB];
    int len, tries = 0;
    SHA256((const unsigned char *)dec, n, digest);
    memset(data, 0, (size_t)f->nb);                                  /* KeyedPRF.pad */
    memcpy(data, digest, f->nb < 32 ? (size_t)f->nb : 32u);
    /* fresh cipher state per eval (util.py:88): reset the CFB-8 register */
    EVP_EncryptInit_ex(f->ctx, NULL, NULL, NULL, zero_iv);
    for (;;) {
        tries++;
        EVP_EncryptUpdate(f->ctx, ct, &len, data, f->nb);            /* stream continues */
        ct[0] &= f->topmask;
        BN_bin2bn(ct, f->nb, out);
        if (BN_cmp(out, f->range) < 0) return tries;
    }
}

/* KeyedPRF.eval(x) for 0 <= x < 2^64. */
static int prf_eval(prf_t *f, uint64_t x, BIGNUM *out) {
    char dec[32];
    int n = snprintf(dec, sizeof dec, "%llu", (unsigned long long)x);   /* str(x) */
    return prf_eval_msg(f, dec, (size_t)n, out);
}

/* prf::evaluate(i) (prf.hxx:125-145) -> out; returns number of tries. */
static int cxx_prf_eval(prf_t *f, uint32_t i, BIGNUM *out) {
    static const unsigned char zero_iv[16] = {0};
    unsigned char digest[32], buf[HBO_MAX_NB], ct[HBO_MAX_NB], le[4];
    int len, tries = 0;
    unsigned count = 0;
    le[0] = (unsigned char)i; le[1] = (unsigned char)(i >> 8);
    le[2] = (unsigned char)(i >> 16); le[3] = (unsigned char)(i >> 24);
    EVP_EncryptInit_ex(f->ctx, NULL, NULL, NULL, zero_iv);          /* Resynchronize */
    for (;;) {
        tries++;
        /* rand_buf (:170-176): memset limit_sz, digest into the buffer */
        SHA256(le, 4, digest);
        memset(buf, 0, (size_t)f->nb);
        memcpy(buf, digest, f->nb < 32 ? (size_t)f->nb : 32u);
        EVP_EncryptUpdate(f->ctx, ct, &len, buf, f->nb);
        ct[0] &= f->topmask;                                            /* SetByte(limit_sz-1, ..) */
        BN_bin2bn(ct, f->nb, out);
        if (!(BN_cmp(out, f->range) >= 0 && count++ < 80)) return tries;
    }
}

/* ------------------------------------------------------------------ API */

int hbo_cxx_prf_eval(const unsigned char *key, size_t keylen,
                     const unsigned char *range_be, size_t range_len,
                     uint32_t x, unsigned char *out_be, size_t out_len) {
    prf_t f;
    BIGNUM *v;
    int tries, rc = prf_init_mode(&f, key, keylen, range_be, range_len, 1);
    if (rc) return rc;
    v = BN_new();
    tries = cxx_prf_eval(&f, x, v);
    BN_bn2binpad(v, out_be, (int)out_len);
    BN_free(v);
    prf_free(&f);
    return tries;
}

int hbo_prf_eval(const unsigned char *key, size_t keylen,
                 const unsigned char *range_be, size_t range_len,
                 uint64_t x, unsigned char *out_be, size_t out_len) {
    prf_t f;
    BIGNUM *v;
    int tries, rc = prf_init(&f, key, keylen, range_be, range_len);
    if (rc) return rc;
    v = BN_new();
    tries = prf_eval(&f, x, v);
    BN_bn2binpad(v, out_be, (int)out_len);
    BN_free(v);
    prf_free(&f);
    return tries;
}

/* KeyedPRF.eval(x) for any Python int x given as its decimal string str(x)
 * (util.py:91 hashes str(x), so negative and > 64-bit inputs are valid). */
int hbo_prf_eval_dec(const unsigned char *key, size_t keylen,
                     const unsigned char *range_be, size_t range_len,
                     const char *dec, unsigned char *out_be, size_t out_len) {
    prf_t f;
    BIGNUM *v;
    int tries, rc = prf_init(&f, key, keylen, range_be, range_len);
    if (rc) return rc;
    v = BN_new();
    tries = prf_eval_msg(&f, dec, strlen(dec), v);
    BN_bn2binpad(v, out_be, (int)out_len);
    BN_free(v);
    prf_free(&f);
    return tries;
}

/* m = BE integer of data[pos : min(pos+ss, len)], 0 if pos >= len.
 * Returns bytes read (the reference breaks out of the sector loop when it is
 * != ss, PySwizzle.py:304-306 / :359-360). */
static uint64_t read_sector(const unsigned char *data, uint64_t len, uint64_t pos,
                            uint64_t ss, BIGNUM *m) {
    uint64_t r;
    if (pos >= len) { BN_zero(m); return 0; }
    r = len - pos < ss ? len - pos : ss;
    BN_bin2bn(data + pos, (int)r, m);
    return r;
}

typedef struct {
    const unsigned char *p_be; size_t p_len;
    uint32_t sectors;
    const unsigned char *f_key, *a_key; size_t keylen;
    uint64_t block_base;
    const unsigned char *data; uint64_t len;
    uint64_t b0, b1;            /* block slice [b0,b1) relative to data */
    unsigned char *tags; int width;
    BIGNUM **alpha;             /* shared, read-only */
    int mode;
    int rc;
} enc_job_t;

static void *encode_worker(void *arg) {
    enc_job_t *J = (enc_job_t *)arg;
    prf_t f;
    BN_CTX *bctx = BN_CTX_new();
    BIGNUM *p = BN_bin2bn(J->p_be, (int)J->p_len, NULL);
    BIGNUM *sigma = BN_new(), *m = BN_new(), *t = BN_new();
    uint64_t ss = (uint64_t)(BN_num_bits(p) / 8), C = ss * J->sectors, i;
    J->rc = prf_init_mode(&f, J->f_key, J->keylen, J->p_be, J->p_len, J->mode);
    if (J->rc) goto out;
    for (i = J->b0; i < J->b1; i++) {
        uint32_t j;
        if (J->mode)   /* s.f(chunk_id), unsigned int chunk_id (shacham_waters_private.cxx:672) */
            cxx_prf_eval(&f, (uint32_t)(J->block_base + i), sigma);
        else
            prf_eval(&f, J->block_base + i, sigma);             /* sigma = f.eval(chunk_id) */
        for (j = 0; j < J->sectors; j++) {
            uint64_t r = read_sector(J->data, J->len, i * C + j * ss, ss, m);
            if (r > 0) {
                BN_mul(t, J->alpha[j], m, bctx);
                BN_add(sigma, sigma, t);
                if (J->mode) BN_mod(sigma, sigma, p, bctx);      /* sigma %= _p (:685) */
            }
            if (r != ss) break;
        }
        if (!J->mode) BN_mod(sigma, sigma, p, bctx);
        BN_bn2binpad(sigma, J->tags + (size_t)(i * (uint64_t)J->width), J->width);
    }
    prf_free(&f);
out:
    BN_free(p); BN_free(sigma); BN_free(m); BN_free(t);
    BN_CTX_free(bctx);
    return NULL;
}

/* Tags for blocks block_base .. block_base+nblocks-1 of `data` (block k of the
 * call starts at data[k*C]; bytes at or past `len` are end of file).  The
 * whole-file PySwizzle encode is block_base = 0, nblocks = len/C + 1.
 * Tags are written big-endian, `width` = ceil(bitlen(p)/8) bytes each. */
static int encode_mode(const unsigned char *p_be, size_t p_len, uint32_t sectors,
                       const unsigned char *f_key, const unsigned char *a_key, size_t keylen,
                       uint64_t block_base, const unsigned char *data, uint64_t len,
                       uint64_t nblocks, unsigned char *tags_out, int nthreads, int mode);

int hbo_encode(const unsigned char *p_be, size_t p_len, uint32_t sectors,
               const unsigned char *f_key, const unsigned char *a_key, size_t keylen,
               uint64_t block_base, const unsigned char *data, uint64_t len,
               uint64_t nblocks, unsigned char *tags_out, int nthreads) {
    return encode_mode(p_be, p_len, sectors, f_key, a_key, keylen, block_base, data, len, nblocks,
                       tags_out, nthreads, 0);
}

/* cxx shacham_waters_private::encode (shacham_waters_private.cxx:638-702)
 * with the cxx prf; same block/sector layout and tag count as hbo_encode. */
int hbo_cxx_encode(const unsigned char *p_be, size_t p_len, uint32_t sectors,
                   const unsigned char *f_key, const unsigned char *a_key, size_t keylen,
                   uint64_t block_base, const unsigned char *data, uint64_t len,
                   uint64_t nblocks, unsigned char *tags_out, int nthreads) {
    return encode_mode(p_be, p_len, sectors, f_key, a_key, keylen, block_base, data, len, nblocks,
                       tags_out, nthreads, 1);
}

static int encode_mode(const unsigned char *p_be, size_t p_len, uint32_t sectors,
                       const unsigned char *f_key, const unsigned char *a_key, size_t keylen,
                       uint64_t block_base, const unsigned char *data, uint64_t len,
                       uint64_t nblocks, unsigned char *tags_out, int nthreads, int mode) {
    BIGNUM *p = BN_bin2bn(p_be, (int)p_len, NULL);
    int bits = BN_num_bits(p), width = (bits + 7) / 8, rc = 0, t;
    BIGNUM **alpha;
    prf_t a;
    pthread_t *th;
    enc_job_t *jobs;
    if (bits < 8 || sectors == 0) { BN_free(p); return -4; }
    alpha = (BIGNUM **)calloc(sectors, sizeof(BIGNUM *));
    rc = prf_init_mode(&a, a_key, keylen, p_be, p_len, mode);
    if (rc) { BN_free(p); free(alpha); return rc; }
    for (uint32_t j = 0; j < sectors; j++) {                 /* alpha.eval(j), PySwizzle.py:302 */
        alpha[j] = BN_new();                                 /* cxx: s.alpha(j), :681 */
        if (mode) cxx_prf_eval(&a, j, alpha[j]);
        else prf_eval(&a, j, alpha[j]);
    }
    prf_free(&a);
    if (nthreads < 1) nthreads = 1;
    if ((uint64_t)nthreads > nblocks) nthreads = (int)(nblocks ? nblocks : 1);
    th = (pthread_t *)calloc((size_t)nthreads, sizeof(pthread_t));
    jobs = (enc_job_t *)calloc((size_t)nthreads, sizeof(enc_job_t));
    for (t = 0; t < nthreads; t++) {
        enc_job_t *J = &jobs[t];
        J->p_be = p_be; J->p_len = p_len; J->sectors = sectors;
        J->f_key = f_key; J->a_key = a_key; J->keylen = keylen;
        J->block_base = block_base; J->data = data; J->len = len;
        J->b0 = nblocks * (uint64_t)t / (uint64_t)nthreads;
        J->b1 = nblocks * (uint64_t)(t + 1) / (uint64_t)nthreads;
        J->tags = tags_out; J->width = width; J->alpha = alpha; J->mode = mode;
        if (nthreads == 1) encode_worker(J);
        else pthread_create(&th[t], NULL, encode_worker, J);
    }
    for (t = 0; t < nthreads; t++) {
        if (nthreads > 1) pthread_join(th[t], NULL);
        if (jobs[t].rc) rc = jobs[t].rc;
    }
    for (uint32_t j = 0; j < sectors; j++) BN_free(alpha[j]);
    free(alpha); free(th); free(jobs); BN_free(p);
    return rc;
}

/* PySwizzle.prove (PySwizzle.py:333-370).  tags: ntags fixed-width BE values. */
int hbo_prove(const unsigned char *p_be, size_t p_len, uint32_t sectors,
              const unsigned char *chal_key, size_t keylen, uint64_t chunks,
              const unsigned char *vmax_be, size_t vmax_len,
              uint64_t ntags, const unsigned char *tags, int tag_width,
              const unsigned char *data, uint64_t len,
              unsigned char *mu_out, unsigned char *sigma_out) {
    BN_CTX *bctx = BN_CTX_new();
    BIGNUM *p = BN_bin2bn(p_be, (int)p_len, NULL);
    BIGNUM *N = BN_new(), *idx = BN_new(), *v = BN_new(), *m = BN_new(), *t = BN_new();
    BIGNUM *sigma = BN_new(), **mu;
    int width = (BN_num_bits(p) + 7) / 8, rc;
    uint64_t ss = (uint64_t)(BN_num_bits(p) / 8), C = ss * sectors, i;
    unsigned char nbe[8];
    prf_t fi, fv;
    for (int k = 0; k < 8; k++) nbe[k] = (unsigned char)(ntags >> (56 - 8 * k));
    rc = prf_init(&fi, chal_key, keylen, nbe, 8);            /* index = KeyedPRF(key, len(tag.sigma)) */
    if (rc) return rc;
    rc = prf_init(&fv, chal_key, keylen, vmax_be, vmax_len); /* v = KeyedPRF(key, v_max) */
    if (rc) { prf_free(&fi); return rc; }
    mu = (BIGNUM **)calloc(sectors, sizeof(BIGNUM *));
    for (uint32_t j = 0; j < sectors; j++) mu[j] = BN_new();
    BN_zero(sigma);
    for (i = 0; i < chunks; i++) {
        uint64_t ix;
        prf_eval(&fi, i, idx);
        prf_eval(&fv, i, v);
        ix = BN_get_word(idx);
        for (uint32_t j = 0; j < sectors; j++) {
            uint64_t r = read_sector(data, len, ix * C + j * ss, ss, m);
            if (r > 0) { BN_mul(t, v, m, bctx); BN_add(mu[j], mu[j], t); }
            if (r != ss) break;
        }
        BN_bin2bn(tags + ix * (uint64_t)tag_width, tag_width, m);
        BN_mul(t, v, m, bctx);
        BN_add(sigma, sigma, t);
    }
    for (uint32_t j = 0; j < sectors; j++) {
        BN_mod(mu[j], mu[j], p, bctx);
        BN_bn2binpad(mu[j], mu_out + (size_t)j * (size_t)width, width);
        BN_free(mu[j]);
    }
    BN_mod(sigma, sigma, p, bctx);
    BN_bn2binpad(sigma, sigma_out, width);
    free(mu);
    prf_free(&fi); prf_free(&fv);
    BN_free(p); BN_free(N); BN_free(idx); BN_free(v); BN_free(m); BN_free(t); BN_free(sigma);
    BN_CTX_free(bctx);
    return 0;
}

/* PySwizzle.verify (PySwizzle.py:372-395) with a decrypted state.
 * Returns 1 if the proof verifies, 0 if not, <0 on error. */
int hbo_verify(const unsigned char *p_be, size_t p_len, uint32_t sectors,
               const unsigned char *f_key, const unsigned char *a_key, size_t keylen,
               uint64_t state_chunks,
               const unsigned char *chal_key, size_t chal_keylen, uint64_t chunks,
               const unsigned char *vmax_be, size_t vmax_len,
               const unsigned char *mu_be, const unsigned char *sigma_be, int width) {
    BN_CTX *bctx = BN_CTX_new();
    BIGNUM *p = BN_bin2bn(p_be, (int)p_len, NULL);
    BIGNUM *rhs = BN_new(), *idx = BN_new(), *v = BN_new(), *fx = BN_new(), *t = BN_new();
    BIGNUM *a = BN_new(), *mu = BN_new(), *sigma;
    unsigned char nbe[8];
    prf_t fi, fv, ff, fa;
    int rc, ok;
    for (int k = 0; k < 8; k++) nbe[k] = (unsigned char)(state_chunks >> (56 - 8 * k));
    if ((rc = prf_init(&fi, chal_key, chal_keylen, nbe, 8))) return rc;
    if ((rc = prf_init(&fv, chal_key, chal_keylen, vmax_be, vmax_len))) return rc;
    if ((rc = prf_init(&ff, f_key, keylen, p_be, p_len))) return rc;
    if ((rc = prf_init(&fa, a_key, keylen, p_be, p_len))) return rc;
    BN_zero(rhs);
    for (uint64_t i = 0; i < chunks; i++) {
        prf_eval(&fi, i, idx);
        prf_eval(&fv, i, v);
        prf_eval(&ff, BN_get_word(idx), fx);
        BN_mul(t, v, fx, bctx);
        BN_add(rhs, rhs, t);
    }
    for (uint32_t j = 0; j < sectors; j++) {
        prf_eval(&fa, j, a);
        BN_bin2bn(mu_be + (size_t)j * (size_t)width, width, mu);
        BN_mul(t, a, mu, bctx);
        BN_add(rhs, rhs, t);
    }
    BN_mod(rhs, rhs, p, bctx);
    sigma = BN_bin2bn(sigma_be, width, NULL);
    ok = BN_cmp(sigma, rhs) == 0;
    prf_free(&fi); prf_free(&fv); prf_free(&ff); prf_free(&fa);
    BN_free(p); BN_free(rhs); BN_free(idx); BN_free(v); BN_free(fx); BN_free(t);
    BN_free(a); BN_free(mu); BN_free(sigma);
    BN_CTX_free(bctx);
    return ok;
}
