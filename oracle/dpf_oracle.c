/*
 * dpf_oracle.c — TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of dkales/dpf-go's evaluation path, used as the parity
 * checker for the HIP engine and as the CPU baseline ("port") in bench.py.
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
 * load this library; the product (dpf-go_amd/) never links or calls it.
 *
 * The reference is Go + Plan-9 amd64 assembly, which cannot be compiled in
 * this image (no go toolchain), so there is no oracle/_ref build.  Parity is
 * pinned by (a) the FIPS-197 AES-128 known answer, (b) fixed-key KATs
 * computed with OpenSSL (tests/golden/aes_kat.json, script committed), and
 * (c) the reference's own property tests (dpf/dpf_test.go:32-73) restated.
 * The reference holds no DPF golden vectors and its Gen draws from
 * crypto/rand (dpf/dpf.go:80-81), so above the AES layer (key layout, CW
 * arithmetic, leaf order) this oracle is PARITY UNPINNED: the properties in
 * (c) are all that ties it to the reference.
 *
 * Each function cites the reference line it follows.  Two AES back ends:
 *   - portable: S-box derived from GF(2^8) inversion + affine map (FIPS-197
 *     §5.1.1), round function written out byte-wise — the checker;
 *   - AES-NI: one block per call, exactly like aes128MMO's AESENC chain
 *     (dpf/aes_amd64.s:51-82) — used as the reference-faithful CPU baseline.
 */
#define _GNU_SOURCE
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <pthread.h>

#if defined(__x86_64__)
#include <immintrin.h>
#include <cpuid.h>
#endif

typedef uint8_t block_t[16];

/* ---------------------------------------------------------------- AES --- */

static uint8_t SBOX[256];
static int g_init = 0;

static uint8_t gf_mul(uint8_t a, uint8_t b) {
    uint8_t p = 0;
    while (b) {
        if (b & 1) p ^= a;
        a = (uint8_t)((a << 1) ^ ((a & 0x80) ? 0x1b : 0));
        b >>= 1;
    }
    return p;
}

static void build_sbox(void) {
    /* FIPS-197 §5.1.1: multiplicative inverse in GF(2^8), then the affine map. */
    for (int x = 0; x < 256; ++x) {
        uint8_t inv = 0;
        if (x) {
            for (int y = 1; y < 256; ++y)
                if (gf_mul((uint8_t)x, (uint8_t)y) == 1) { inv = (uint8_t)y; break; }
        }
        uint8_t s = inv;
        uint8_t r = inv;
        for (int i = 0; i < 4; ++i) {
            r = (uint8_t)((r << 1) | (r >> 7));
            s ^= r;
        }
        SBOX[x] = (uint8_t)(s ^ 0x63);
    }
}

/* Standard AES-128 key schedule — what expandKeyAsm/_expand_key_128 compute
 * (dpf/aes_amd64.s:87-126, rcon 01..36 at :95-114).  11 round keys, 16 B
 * each, in byte order. */
void oracle_expand_key(const uint8_t key[16], uint8_t rk[176]) {
    static const uint8_t rcon[10] = {0x01, 0x02, 0x04, 0x08, 0x10, 0x20, 0x40, 0x80, 0x1b, 0x36};
    memcpy(rk, key, 16);
    for (int i = 4; i < 44; ++i) {
        uint8_t t[4];
        memcpy(t, rk + 4 * (i - 1), 4);
        if (i % 4 == 0) {
            uint8_t u = t[0];
            t[0] = (uint8_t)(SBOX[t[1]] ^ rcon[i / 4 - 1]);
            t[1] = SBOX[t[2]];
            t[2] = SBOX[t[3]];
            t[3] = SBOX[u];
        }
        for (int j = 0; j < 4; ++j) rk[4 * i + j] = (uint8_t)(rk[4 * (i - 4) + j] ^ t[j]);
    }
}

static uint8_t xtime(uint8_t a) { return (uint8_t)((a << 1) ^ ((a & 0x80) ? 0x1b : 0)); }

/* Plain AES-128 encryption of one block (FIPS-197 §5.1); byte index 4c+r is
 * row r of column c, matching MOVUPS loads of a [16]byte (aes_amd64.s:56). */
void oracle_aes128_encrypt(const uint8_t rk[176], uint8_t out[16], const uint8_t in[16]) {
    uint8_t s[16], t[16];
    for (int i = 0; i < 16; ++i) s[i] = (uint8_t)(in[i] ^ rk[i]);
    for (int round = 1; round <= 10; ++round) {
        for (int i = 0; i < 16; ++i) s[i] = SBOX[s[i]];
        for (int c = 0; c < 4; ++c)          /* ShiftRows: row r rotates left by r */
            for (int r = 0; r < 4; ++r) t[4 * c + r] = s[4 * ((c + r) & 3) + r];
        if (round != 10) {
            for (int c = 0; c < 4; ++c) {    /* MixColumns */
                uint8_t a0 = t[4 * c], a1 = t[4 * c + 1], a2 = t[4 * c + 2], a3 = t[4 * c + 3];
                uint8_t all = (uint8_t)(a0 ^ a1 ^ a2 ^ a3);
                s[4 * c + 0] = (uint8_t)(a0 ^ all ^ xtime((uint8_t)(a0 ^ a1)));
                s[4 * c + 1] = (uint8_t)(a1 ^ all ^ xtime((uint8_t)(a1 ^ a2)));
                s[4 * c + 2] = (uint8_t)(a2 ^ all ^ xtime((uint8_t)(a2 ^ a3)));
                s[4 * c + 3] = (uint8_t)(a3 ^ all ^ xtime((uint8_t)(a3 ^ a0)));
            }
        } else {
            memcpy(s, t, 16);
        }
        for (int i = 0; i < 16; ++i) s[i] ^= rk[16 * round + i];
    }
    memcpy(out, s, 16);
}

/* --------------------------------------------------------- PRG keys --- */

/* dpf/dpf.go:23-24 */
static const uint8_t PRFKEY_L[16] = {36, 156, 50, 234, 92, 230, 49, 9, 174, 170, 205, 160, 98, 236, 29, 243};
static const uint8_t PRFKEY_R[16] = {209, 12, 199, 173, 29, 74, 44, 128, 194, 224, 14, 44, 2, 201, 110, 28};
static uint8_t RK_L[176], RK_R[176];
static int g_have_aesni = 0;

static int detect_aesni(void) {
#if defined(__x86_64__)
    unsigned a, b, c, d;
    if (!__get_cpuid(1, &a, &b, &c, &d)) return 0;
    return (c & bit_AES) != 0;
#else
    return 0;
#endif
}

/* dpf/dpf.go:22-44 (init): expand keyL / keyR once. */
void oracle_init(void) {
    if (g_init) return;
    build_sbox();
    oracle_expand_key(PRFKEY_L, RK_L);
    oracle_expand_key(PRFKEY_R, RK_R);
    g_have_aesni = detect_aesni();
    g_init = 1;
}

int oracle_have_aesni(void) { oracle_init(); return g_have_aesni; }
const uint8_t* oracle_round_keys(int right) { oracle_init(); return right ? RK_R : RK_L; }

/* aes128MMO (dpf/aes_amd64.s:51-82): dst = AES_k(src) XOR src, dst may alias src. */
typedef void (*mmo_fn)(const uint8_t* rk, uint8_t* dst, const uint8_t* src);

static void mmo_portable(const uint8_t* rk, uint8_t* dst, const uint8_t* src) {
    uint8_t e[16];
    oracle_aes128_encrypt(rk, e, src);
    for (int i = 0; i < 16; ++i) dst[i] = (uint8_t)(e[i] ^ src[i]);
}

#if defined(__x86_64__)
__attribute__((target("aes,sse2")))
static void mmo_aesni(const uint8_t* rk, uint8_t* dst, const uint8_t* src) {
    /* One block per call with the serial AESENC chain, as the reference does. */
    __m128i x = _mm_loadu_si128((const __m128i*)src);
    __m128i s = _mm_xor_si128(x, _mm_loadu_si128((const __m128i*)rk));
    for (int r = 1; r < 10; ++r) s = _mm_aesenc_si128(s, _mm_loadu_si128((const __m128i*)(rk + 16 * r)));
    s = _mm_aesenclast_si128(s, _mm_loadu_si128((const __m128i*)(rk + 160)));
    _mm_storeu_si128((__m128i*)dst, _mm_xor_si128(s, x));
}
#endif

static mmo_fn pick_mmo(int use_aesni) {
    oracle_init();
#if defined(__x86_64__)
    if (use_aesni && g_have_aesni) return mmo_aesni;
#endif
    (void)use_aesni;
    return mmo_portable;
}

void oracle_mmo(int right, int use_aesni, uint8_t* dst, const uint8_t* src) {
    mmo_fn f = pick_mmo(use_aesni);
    f(right ? RK_R : RK_L, dst, src);
}

/* ------------------------------------------------------------- DPF --- */

static void xor16(uint8_t* dst, const uint8_t* a, const uint8_t* b) {     /* aes_amd64.s:8-16 */
    for (int i = 0; i < 16; ++i) dst[i] = (uint8_t)(a[i] ^ b[i]);
}
static uint8_t getT(const uint8_t* in) { return (uint8_t)(*in & 1); }   /* dpf.go:46-48 */
static void clr(uint8_t* in) { *in &= (uint8_t)~1u; }                  /* dpf.go:50-52 */

/* prg (dpf/dpf.go:59-69) */
static void prg(mmo_fn f, const uint8_t* seed, uint8_t* s0, uint8_t* s1, uint8_t* t0, uint8_t* t1) {
    f(RK_L, s0, seed);
    *t0 = getT(s0);
    clr(s0);
    f(RK_R, s1, seed);
    *t1 = getT(s1);
    clr(s1);
}

static uint64_t stop_of(uint64_t logN) { return logN >= 7 ? logN - 7 : 0; }

size_t oracle_key_len(uint64_t logN) { return 33 + 18 * (size_t)stop_of(logN); }
size_t oracle_out_len(uint64_t logN) { return logN >= 7 ? ((size_t)1 << (logN - 3)) : 16; }

/* Gen (dpf/dpf.go:71-169) with s0/s1 injected instead of crypto/rand (:80-81).
 * Returns -1 where the reference panics (:72-74). ka/kb: oracle_key_len bytes. */
int oracle_gen(uint64_t alpha, uint64_t logN, const uint8_t seed0[16], const uint8_t seed1[16],
               uint8_t* ka, uint8_t* kb) {
    oracle_init();
    if (logN > 63 || alpha >= ((uint64_t)1 << logN)) return -1;
    mmo_fn f = pick_mmo(0);
    block_t s0, s1, scw, s0L, s0R, s1L, s1R;
    memcpy(s0, seed0, 16);
    memcpy(s1, seed1, 16);
    uint8_t t0 = getT(&s0[0]);
    uint8_t t1 = (uint8_t)(t0 ^ 1);
    clr(&s0[0]);
    clr(&s1[0]);
    memcpy(ka, s0, 16); ka[16] = t0;
    memcpy(kb, s1, 16); kb[16] = t1;
    size_t off = 17;
    uint64_t stop = stop_of(logN);
    for (uint64_t i = 0; i < stop; ++i) {
        uint8_t t0L, t0R, t1L, t1R;
        prg(f, s0, s0L, s0R, &t0L, &t0R);
        prg(f, s1, s1L, s1R, &t1L, &t1R);
        if (alpha & ((uint64_t)1 << (logN - 1 - i))) {           /* KEEP = R (:106-131) */
            xor16(scw, s0L, s1L);
            uint8_t tLCW = (uint8_t)(t0L ^ t1L);
            uint8_t tRCW = (uint8_t)(t0R ^ t1R ^ 1);
            memcpy(ka + off, scw, 16); ka[off + 16] = tLCW; ka[off + 17] = tRCW;
            memcpy(s0, s0R, 16);
            if (t0) xor16(s0, s0, scw);
            memcpy(s1, s1R, 16);
            if (t1) xor16(s1, s1, scw);
            t0 = t0 ? (uint8_t)(t0R ^ tRCW) : t0R;
            t1 = t1 ? (uint8_t)(t1R ^ tRCW) : t1R;
        } else {                                                   /* KEEP = L (:132-157) */
            xor16(scw, s0R, s1R);
            uint8_t tLCW = (uint8_t)(t0L ^ t1L ^ 1);
            uint8_t tRCW = (uint8_t)(t0R ^ t1R);
            memcpy(ka + off, scw, 16); ka[off + 16] = tLCW; ka[off + 17] = tRCW;
            memcpy(s0, s0L, 16);
            if (t0) xor16(s0, s0, scw);
            memcpy(s1, s1L, 16);
            if (t1) xor16(s1, s1, scw);
            t0 = t0 ? (uint8_t)(t0L ^ tLCW) : t0L;
            t1 = t1 ? (uint8_t)(t1L ^ tLCW) : t1L;
        }
        off += 18;
    }
    f(RK_L, s0, s0);                                               /* :160 */
    f(RK_L, s1, s1);                                               /* :162 */
    xor16(scw, s0, s1);                                            /* :163 */
    scw[(alpha & 127) / 8] ^= (uint8_t)(1u << ((alpha & 127) % 8)); /* :164 */
    memcpy(ka + off, scw, 16);                                     /* :165-167 */
    memcpy(kb + 17, ka + 17, off - 17);
    memcpy(kb + off, scw, 16);
    return 0;
}

/* Eval (dpf/dpf.go:171-211).  Reads the final CW at len(k)-16 (:206). */
static uint8_t eval_with(mmo_fn f, const uint8_t* k, size_t klen, uint64_t x, uint64_t logN) {
    block_t s, sL, sR;
    memcpy(s, k, 16);                                              /* :175, no LSB clear */
    uint8_t t = k[16];
    uint64_t stop = stop_of(logN);
    for (uint64_t i = 0; i < stop; ++i) {
        uint8_t tL, tR;
        prg(f, s, sL, sR, &tL, &tR);
        if (t != 0) {                                              /* :185-193 */
            const uint8_t* sCW = k + 17 + i * 18;
            xor16(sL, sL, sCW);
            xor16(sR, sR, sCW);
            tL ^= k[17 + i * 18 + 16];
            tR ^= k[17 + i * 18 + 17];
        }
        /* :194 -- Go's `uint64(1) << n` is 0 for n >= 64 (C leaves it undefined) */
        uint64_t sh = logN - 1 - i, m = sh < 64 ? (uint64_t)1 << sh : 0;
        if (x & m)                                { memcpy(s, sR, 16); t = tR; }
        else                                      { memcpy(s, sL, 16); t = tL; }
    }
    f(RK_L, s, s);                                                 /* :204 */
    if (t != 0) xor16(s, s, k + klen - 16);                        /* :205-206 */
    return (uint8_t)((s[(x & 127) / 8] >> ((x & 127) % 8)) & 1);   /* :207/:209 */
}

int oracle_eval(const uint8_t* k, size_t klen, uint64_t x, uint64_t logN, int use_aesni) {
    return eval_with(pick_mmo(use_aesni), k, klen, x, logN);
}

/* evalFullRecursive (dpf/dpf.go:213-241): DFS, left before right, leaves
 * appended at a 16-byte cursor. */
typedef struct { uint8_t* data; size_t index; } bytearr;

static void eval_full_rec(mmo_fn f, block_t (*stack)[2], const uint8_t* k, size_t klen,
                          const uint8_t* s, uint8_t t, uint64_t lvl, uint64_t stop, bytearr* res) {
    if (lvl == stop) {
        uint8_t* ss = stack[lvl][0];
        memcpy(ss, s, 16);
        f(RK_L, ss, ss);                                           /* :217 */
        if (t != 0) xor16(res->data + res->index, ss, k + klen - 16);          /* :218-220 */
        else        xor16(res->data + res->index, ss, res->data + res->index); /* :221-223 */
        res->index += 16;
        return;
    }
    uint8_t* sL = stack[lvl][0];
    uint8_t* sR = stack[lvl][1];
    uint8_t tL, tR;
    prg(f, s, sL, sR, &tL, &tR);                                   /* :229 */
    if (t != 0) {                                                  /* :230-238 */
        const uint8_t* sCW = k + 17 + lvl * 18;
        xor16(sL, sL, sCW);
        xor16(sR, sR, sCW);
        tL ^= k[17 + lvl * 18 + 16];
        tR ^= k[17 + lvl * 18 + 17];
    }
    eval_full_rec(f, stack, k, klen, sL, tL, lvl + 1, stop, res);  /* :239 */
    eval_full_rec(f, stack, k, klen, sR, tR, lvl + 1, stop, res);  /* :240 */
}

/* EvalFull (dpf/dpf.go:243-262).  out must hold oracle_out_len(logN) bytes;
 * it is zero-filled first, as Go's make() does (:248/:251). */
static void evalfull_with(mmo_fn f, const uint8_t* key, size_t klen, uint64_t logN, uint8_t* out) {
    block_t s;
    memcpy(s, key, 16);
    uint8_t t = key[16];
    uint64_t stop = stop_of(logN);
    memset(out, 0, oracle_out_len(logN));
    bytearr b = {out, 0};
    block_t stack[64][2];
    eval_full_rec(f, stack, key, klen, s, t, 0, stop, &b);
}

void oracle_evalfull(const uint8_t* key, size_t klen, uint64_t logN, uint8_t* out, int use_aesni) {
    evalfull_with(pick_mmo(use_aesni), key, klen, logN, out);
}

/* Batched drivers for the CPU baseline: keys split over nthreads POSIX
 * threads, one key per thread at a time — the equivalent of running the
 * reference EvalFull in parallel goroutines. */
typedef struct {
    mmo_fn f;
    const uint8_t* keys; size_t klen; size_t nkeys; uint64_t logN; uint8_t* out;
    const uint64_t* xs; size_t pts; int nthreads, tid;
} job_t;

static void* evalfull_worker(void* p) {
    job_t* j = (job_t*)p;
    size_t ol = oracle_out_len(j->logN);
    for (size_t k = (size_t)j->tid; k < j->nkeys; k += (size_t)j->nthreads)
        evalfull_with(j->f, j->keys + k * j->klen, j->klen, j->logN, j->out + k * ol);
    return NULL;
}

static void* eval_worker(void* p) {
    job_t* j = (job_t*)p;
    for (size_t k = (size_t)j->tid; k < j->nkeys; k += (size_t)j->nthreads)
        for (size_t q = 0; q < j->pts; ++q)
            j->out[k * j->pts + q] = eval_with(j->f, j->keys + k * j->klen, j->klen,
                                               j->xs[k * j->pts + q], j->logN);
    return NULL;
}

static void run_jobs(job_t* base, void* (*fn)(void*)) {
    int n = base->nthreads < 1 ? 1 : base->nthreads;
    if (n > 256) n = 256;
    pthread_t th[256];
    job_t jobs[256];
    for (int i = 0; i < n; ++i) { jobs[i] = *base; jobs[i].nthreads = n; jobs[i].tid = i; }
    for (int i = 1; i < n; ++i) pthread_create(&th[i], NULL, fn, &jobs[i]);
    fn(&jobs[0]);
    for (int i = 1; i < n; ++i) pthread_join(th[i], NULL);
}

void oracle_evalfull_batch(const uint8_t* keys, size_t klen, size_t nkeys, uint64_t logN,
                           uint8_t* out, int nthreads, int use_aesni) {
    job_t j = {pick_mmo(use_aesni), keys, klen, nkeys, logN, out, NULL, 0, nthreads, 0};
    run_jobs(&j, evalfull_worker);
}

void oracle_eval_batch(const uint8_t* keys, size_t klen, size_t nkeys, const uint64_t* xs,
                       size_t pts_per_key, uint64_t logN, uint8_t* out, int nthreads, int use_aesni) {
    job_t j = {pick_mmo(use_aesni), keys, klen, nkeys, logN, out, xs, pts_per_key, nthreads, 0};
    run_jobs(&j, eval_worker);
}

/* EvalFull of one key on nthreads threads, for the full-size parity checks
 * (configs[3]: logN = 32, 512 MiB).  The DFS (dpf.go:213-241) visits left
 * before right, so the output is the concatenation of the 2^d subtrees at
 * depth d in prefix order.  Thread j takes subtrees j, j+n, ...: it walks the
 * root to subtree p's root with the same per-level step evalFullRecursive
 * applies (prg + CW under t, :229-238, child chosen by bit d-1-i of p) and
 * then runs the recursion from level d into the subtree's slice of out. */
typedef struct {
    mmo_fn f;
    const uint8_t* key; size_t klen; uint64_t logN; uint8_t* out;
    int depth, nthreads, tid;
} sub_job_t;

static void* evalfull_sub_worker(void* p) {
    sub_job_t* j = (sub_job_t*)p;
    uint64_t stop = stop_of(j->logN);
    size_t part = oracle_out_len(j->logN) >> j->depth;
    block_t stack[64][2];
    for (uint64_t pre = (uint64_t)j->tid; pre < ((uint64_t)1 << j->depth); pre += (uint64_t)j->nthreads) {
        block_t s, sL, sR;
        memcpy(s, j->key, 16);
        uint8_t t = j->key[16];
        for (int i = 0; i < j->depth; ++i) {
            uint8_t tL, tR;
            prg(j->f, s, sL, sR, &tL, &tR);
            if (t != 0) {
                const uint8_t* sCW = j->key + 17 + (size_t)i * 18;
                xor16(sL, sL, sCW);
                xor16(sR, sR, sCW);
                tL ^= j->key[17 + i * 18 + 16];
                tR ^= j->key[17 + i * 18 + 17];
            }
            if ((pre >> (j->depth - 1 - i)) & 1) { memcpy(s, sR, 16); t = tR; }
            else                                 { memcpy(s, sL, 16); t = tL; }
        }
        bytearr b = {j->out + pre * part, 0};
        eval_full_rec(j->f, stack, j->key, j->klen, s, t, (uint64_t)j->depth, stop, &b);
    }
    return NULL;
}

void oracle_evalfull_mt(const uint8_t* key, size_t klen, uint64_t logN, uint8_t* out, int nthreads,
                        int use_aesni) {
    mmo_fn f = pick_mmo(use_aesni);
    uint64_t stop = stop_of(logN);
    int n = nthreads < 1 ? 1 : (nthreads > 256 ? 256 : nthreads);
    int depth = 0;
    while (depth < 8 && (uint64_t)depth < stop && (1 << depth) < 4 * n) ++depth;
    memset(out, 0, oracle_out_len(logN));
    if (depth == 0) { evalfull_with(f, key, klen, logN, out); return; }
    if (n > (1 << depth)) n = 1 << depth;
    pthread_t th[256];
    sub_job_t jobs[256];
    for (int i = 0; i < n; ++i) {
        sub_job_t jj = {f, key, klen, logN, out, depth, n, i};
        jobs[i] = jj;
    }
    for (int i = 1; i < n; ++i) pthread_create(&th[i], NULL, evalfull_sub_worker, &jobs[i]);
    evalfull_sub_worker(&jobs[0]);
    for (int i = 1; i < n; ++i) pthread_join(th[i], NULL);
}

/* PIR answer (build-only operator, SURVEY §8a last row): XOR of the 32-byte
 * DB records whose EvalFull bit is set.  Records [rec_lo, rec_lo+nrec). */
void oracle_pir_answer(const uint8_t* key, size_t klen, uint64_t logN, const uint8_t* db,
                       uint64_t rec_lo, uint64_t nrec, uint8_t ans[32]) {
    size_t ol = oracle_out_len(logN);
    uint8_t* bits = (uint8_t*)malloc(ol);
    oracle_evalfull(key, klen, logN, bits, 1);
    memset(ans, 0, 32);
    for (uint64_t i = 0; i < nrec; ++i) {
        uint64_t x = rec_lo + i;
        if ((bits[x >> 3] >> (x & 7)) & 1)
            for (int b = 0; b < 32; ++b) ans[b] ^= db[i * 32 + b];
    }
    free(bits);
}

/* The same answer for a batch of keys, split into nslices equal record
 * slices of the domain (slice s = records [s*2^logN/nslices, (s+1)*...) of
 * the DB, cut at nrec): ans[k][s][32] is key k's partial over slice s, the
 * value an N = nslices PIR rank returns; XOR over s gives oracle_pir_answer.
 * Keys are split over nthreads threads; each key's EvalFull bits
 * (dpf.go:243-262, AES-NI restatement) select records by a 64-bit mask
 * instead of a branch, XORed 8 bytes at a time. */
typedef struct {
    const uint8_t* keys; size_t klen; size_t nkeys; uint64_t logN;
    const uint8_t* db; uint64_t nrec; int nslices; uint8_t* ans; int nthreads, tid;
} pir_job_t;

static void* pir_worker(void* p) {
    pir_job_t* j = (pir_job_t*)p;
    size_t ol = oracle_out_len(j->logN);
    uint8_t* bits = (uint8_t*)malloc(ol);
    uint64_t dom = j->logN >= 64 ? ~(uint64_t)0 : ((uint64_t)1 << j->logN);
    uint64_t per = dom / (uint64_t)j->nslices;
    for (size_t k = (size_t)j->tid; k < j->nkeys; k += (size_t)j->nthreads) {
        evalfull_with(pick_mmo(1), j->keys + k * j->klen, j->klen, j->logN, bits);
        for (int s = 0; s < j->nslices; ++s) {
            uint64_t lo = (uint64_t)s * per, hi = lo + per;
            if (hi > j->nrec) hi = j->nrec;
            uint64_t acc[4] = {0, 0, 0, 0};
            for (uint64_t x = lo; x < hi; ++x) {
                uint64_t m = (uint64_t)0 - (uint64_t)((bits[x >> 3] >> (x & 7)) & 1);
                uint64_t r[4];
                memcpy(r, j->db + x * 32, 32);
                acc[0] ^= r[0] & m; acc[1] ^= r[1] & m; acc[2] ^= r[2] & m; acc[3] ^= r[3] & m;
            }
            memcpy(j->ans + (k * (size_t)j->nslices + (size_t)s) * 32, acc, 32);
        }
    }
    free(bits);
    return NULL;
}

void oracle_pir_answer_batch(const uint8_t* keys, size_t klen, size_t nkeys, uint64_t logN, const uint8_t* db,
                             uint64_t nrec, int nslices, uint8_t* ans, int nthreads) {
    oracle_init();
    int n = nthreads < 1 ? 1 : (nthreads > 256 ? 256 : nthreads);
    if (nslices < 1) nslices = 1;
    pthread_t th[256];
    pir_job_t jobs[256];
    for (int i = 0; i < n; ++i) {
        pir_job_t jj = {keys, klen, nkeys, logN, db, nrec, nslices, ans, n, i};
        jobs[i] = jj;
    }
    for (int i = 1; i < n; ++i) pthread_create(&th[i], NULL, pir_worker, &jobs[i]);
    pir_worker(&jobs[0]);
    for (int i = 1; i < n; ++i) pthread_join(th[i], NULL);
}
