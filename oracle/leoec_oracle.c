/*
 * leoec_oracle.c — CPU restatement of leo_erasure's coding path.
 *
 * TEST INFRASTRUCTURE ONLY (see leoec_oracle.h).  The product never links,
 * loads or calls anything in this file.
 *
 * Every function cites the reference call site it restates.  The arithmetic
 * libraries (gf-complete, Jerasure fork, ISA-L fork) are git-cloned unpinned
 * at build time by c_src/build_deps.sh:48-60 and are absent here; their
 * published algorithms (Jerasure 2.0 / gf-complete 1.0 / ISA-L 2.x) are
 * restated from the public documentation and pinned by tests/test_oracle.py.
 */
#define _GNU_SOURCE
#include "leoec_oracle.h"

#include <math.h>
#include <pthread.h>
#include <stdio.h>
#include <sched.h>
#include <time.h>
#include <stdlib.h>
#include <string.h>
#if defined(__x86_64__)
#include <immintrin.h>
#endif

/* ------------------------------------------------------------------------ */
/* Field: gf-complete default primitive polynomials (the octal table shared
 * with Jerasure 1.2's galois.c; gf_w4/w8/w16/w32 defaults coincide).
 * Used by galois_init_default_field_noalloc (c_src/leo_erasure_nif.cpp:124-126)
 * and galois_single_multiply/divide inside Jerasure.                        */
static const uint64_t kPoly[33] = {
    0,           01,          07,          013,         023,
    045,         0103,        0211,        0435,        01021,
    02011,       04005,       010123,      020033,      042103,
    0100003,     0210013,     0400011,     01000201,    02000047,
    04000011,    010000005,   020000003,   040000041,   0100000207,
    0200000011,  0400000107,  01000000047, 02000000011, 04000000005,
    010040000007, 020000000011, 00020000007 /* w=32: x^32 implicit */};

uint64_t orc_prim_poly(int w) {
  if (w < 1 || w > 32) return 0;
  if (w == 32) return (1ull << 32) | kPoly[32];
  return kPoly[w];
}

uint32_t orc_gf_mul(uint32_t a, uint32_t b, int w) {
  if (w == 1) return a & b & 1;
  uint64_t poly = orc_prim_poly(w);
  uint64_t r = 0;
  for (int i = 0; i < w; i++)
    if ((b >> i) & 1) r ^= (uint64_t)a << i;
  for (int i = 2 * w - 2; i >= w; i--)
    if ((r >> i) & 1) r ^= poly << (i - w);
  return (uint32_t)r;
}

uint32_t orc_gf_inv(uint32_t a, int w) {
  if (a == 0) return 0;
  /* a^(2^w - 2) */
  uint64_t e = (w == 32) ? 0xFFFFFFFEull : ((1ull << w) - 2);
  uint32_t r = 1, base = a;
  while (e) {
    if (e & 1) r = orc_gf_mul(r, base, w);
    base = orc_gf_mul(base, base, w);
    e >>= 1;
  }
  return r;
}

uint32_t orc_gf_div(uint32_t a, uint32_t b, int w) {
  if (b == 0) return (uint32_t)-1; /* galois_single_divide(a, 0) returns -1 */
  if (a == 0) return 0;
  return orc_gf_mul(a, orc_gf_inv(b, w), w);
}

/* ------------------------------------------------------------------------ */
/* Jerasure reed_sol_extended_vandermonde_matrix +
 * reed_sol_big_vandermonde_distribution_matrix +
 * reed_sol_vandermonde_coding_matrix (called c_src/rscoding.cpp:67,143,194). */
static uint32_t *ext_vandermonde(int rows, int cols, int w) {
  if (w < 30 && ((1ll << w) < rows || (1ll << w) < cols)) return NULL;
  uint32_t *v = calloc((size_t)rows * cols, sizeof(uint32_t));
  if (!v) return NULL;
  v[0] = 1;
  if (rows == 1) return v;
  v[(size_t)(rows - 1) * cols + cols - 1] = 1;
  if (rows == 2) return v;
  for (int i = 1; i < rows - 1; i++) {
    uint32_t p = 1;
    for (int j = 0; j < cols; j++) {
      v[(size_t)i * cols + j] = p;
      p = orc_gf_mul(p, (uint32_t)i, w);
    }
  }
  return v;
}

static uint32_t *big_vandermonde_distribution(int rows, int cols, int w) {
  if (cols >= rows) return NULL;
  uint32_t *d = ext_vandermonde(rows, cols, w);
  if (!d) return NULL;
#define D(r, c) d[(size_t)(r) * cols + (c)]
  for (int i = 1; i < cols; i++) {
    int j = i;
    while (j < rows && D(j, i) == 0) j++;
    if (j >= rows) { free(d); return NULL; }
    if (j != i)
      for (int c = 0; c < cols; c++) { uint32_t t = D(i, c); D(i, c) = D(j, c); D(j, c) = t; }
    if (D(i, i) != 1) {
      uint32_t inv = orc_gf_div(1, D(i, i), w);
      for (int r = 0; r < rows; r++) D(r, i) = orc_gf_mul(inv, D(r, i), w);
    }
    for (int c = 0; c < cols; c++) {
      uint32_t e = D(i, c);
      if (c != i && e != 0)
        for (int r = 0; r < rows; r++) D(r, c) ^= orc_gf_mul(e, D(r, i), w);
    }
  }
  /* row `cols` all ones: scale coding part of each column */
  for (int c = 0; c < cols; c++) {
    uint32_t t = D(cols, c);
    if (t != 1) {
      uint32_t inv = orc_gf_div(1, t, w);
      for (int r = cols; r < rows; r++) D(r, c) = orc_gf_mul(inv, D(r, c), w);
    }
  }
  /* first column of each later coding row = 1 */
  for (int r = cols + 1; r < rows; r++) {
    uint32_t t = D(r, 0);
    if (t != 1) {
      uint32_t inv = orc_gf_div(1, t, w);
      for (int c = 0; c < cols; c++) D(r, c) = orc_gf_mul(D(r, c), inv, w);
    }
  }
#undef D
  return d;
}

int orc_vandermonde_coding_matrix(int k, int m, int w, uint32_t *out) {
  uint32_t *d = big_vandermonde_distribution(k + m, k, w);
  if (!d) return ORC_E_UNSUPPORTED;
  memcpy(out, d + (size_t)k * k, sizeof(uint32_t) * (size_t)m * k);
  free(d);
  return ORC_OK;
}

/* ------------------------------------------------------------------------ */
/* Jerasure cauchy.c: cauchy_original_coding_matrix, cauchy_n_ones,
 * cauchy_improve_coding_matrix, cauchy_good_general_coding_matrix
 * (called c_src/cauchycoding.cpp:38,147,197).                              */
int orc_cauchy_original_coding_matrix(int k, int m, int w, uint32_t *out) {
  if (w < 31 && (long long)(k + m) > (1ll << w)) return ORC_E_UNSUPPORTED;
  for (int i = 0; i < m; i++)
    for (int j = 0; j < k; j++)
      out[i * k + j] = orc_gf_div(1, (uint32_t)(i ^ (m + j)), w);
  return ORC_OK;
}

int orc_cauchy_n_ones(uint32_t n, int w) {
  /* total ones of the w x w bitmatrix of n: sum over x of popcount(n * 2^x) */
  int no = 0;
  for (int x = 0; x < w; x++) {
    no += __builtin_popcount(n);
    n = orc_gf_mul(n, 2, w);
  }
  return no;
}

void orc_cauchy_improve_coding_matrix(int k, int m, int w, uint32_t *mat) {
  for (int j = 0; j < k; j++) {
    if (mat[j] != 1) {
      uint32_t t = orc_gf_div(1, mat[j], w);
      for (int i = 0; i < m; i++) mat[i * k + j] = orc_gf_mul(mat[i * k + j], t, w);
    }
  }
  for (int i = 1; i < m; i++) {
    uint32_t *row = mat + (size_t)i * k;
    int bno = 0;
    for (int j = 0; j < k; j++) bno += orc_cauchy_n_ones(row[j], w);
    int bidx = -1;
    for (int j = 0; j < k; j++) {
      if (row[j] != 1) {
        uint32_t t = orc_gf_div(1, row[j], w);
        int tno = 0;
        for (int x = 0; x < k; x++) tno += orc_cauchy_n_ones(orc_gf_mul(row[x], t, w), w);
        if (tno < bno) { bno = tno; bidx = j; }
      }
    }
    if (bidx != -1) {
      uint32_t t = orc_gf_div(1, row[bidx], w);
      for (int j = 0; j < k; j++) row[j] = orc_gf_mul(row[j], t, w);
    }
  }
}

/* cbest_w tables (Jerasure cauchy_best_r6.c) are not available.  They are
 * the nonzero field elements ordered by bitmatrix weight, ties by value: this
 * rule reproduces the recalled cbest_2..cbest_5 exactly (tests pin it).  The
 * max-k bound for w >= 12 is uncertain (recalled as 1023); w > 20 is refused. */
static long cbest_max_k(int w) {
  if (w < 2) return -1;
  if (w <= 11) return (1l << w) - 1;
  return 1023;
}

typedef struct { uint32_t e; int ones; } orc_cb;
static int cb_cmp(const void *a, const void *b) {
  const orc_cb *x = a, *y = b;
  if (x->ones != y->ones) return x->ones < y->ones ? -1 : 1;
  return x->e < y->e ? -1 : (x->e > y->e);
}

int orc_cbest_row(int w, int k, uint32_t *out) {
  if (w < 2 || w > 20 || k > cbest_max_k(w)) return ORC_E_UNSUPPORTED;
  size_t n = ((size_t)1 << w) - 1;
  orc_cb *v = malloc(n * sizeof(orc_cb));
  if (!v) return ORC_E_NOMEM;
  for (size_t i = 0; i < n; i++) { v[i].e = (uint32_t)(i + 1); v[i].ones = orc_cauchy_n_ones(v[i].e, w); }
  qsort(v, n, sizeof(orc_cb), cb_cmp);
  for (int i = 0; i < k; i++) out[i] = v[i].e;
  free(v);
  return ORC_OK;
}

int orc_cauchy_good_general_coding_matrix(int k, int m, int w, uint32_t *out) {
  if (m == 2 && k <= cbest_max_k(w)) {
    for (int i = 0; i < k; i++) out[i] = 1;
    return orc_cbest_row(w, k, out + k);
  }
  int rc = orc_cauchy_original_coding_matrix(k, m, w, out);
  if (rc) return rc;
  orc_cauchy_improve_coding_matrix(k, m, w, out);
  return ORC_OK;
}

/* Jerasure liberation.c liberation_coding_bitmatrix
 * (called c_src/liberationcoding.cpp:39,146,194).  out: 2w rows x kw cols. */
int orc_liberation_coding_bitmatrix(int k, int w, uint8_t *out) {
  if (k > w) return ORC_E_UNSUPPORTED;
  int cols = k * w;
  memset(out, 0, (size_t)2 * w * cols);
  for (int i = 0; i < w; i++)
    for (int j = 0; j < k; j++) out[i * cols + j * w + i] = 1;
  for (int j = 0; j < k; j++) {
    for (int i = 0; i < w; i++) out[(w + i) * cols + j * w + (j + i) % w] = 1;
    if (j > 0) {
      int i = (j * ((w - 1) / 2)) % w;
      out[(w + i) * cols + j * w + (i + j - 1) % w] = 1;
    }
  }
  return ORC_OK;
}

/* Jerasure jerasure_matrix_to_bitmatrix (c_src/cauchycoding.cpp:39). */
int orc_matrix_to_bitmatrix(int k, int m, int w, const uint32_t *mat, uint8_t *out) {
  int cols = k * w;
  for (int i = 0; i < m; i++)
    for (int j = 0; j < k; j++) {
      uint32_t e = mat[i * k + j];
      for (int x = 0; x < w; x++) {
        for (int l = 0; l < w; l++) out[(size_t)(i * w + l) * cols + j * w + x] = (e >> l) & 1;
        e = orc_gf_mul(e, 2, w);
      }
    }
  return ORC_OK;
}

/* ISA-L gf_gen_cauchy1_matrix (c_src/irscoding.cpp:68,131,173). */
int orc_isal_gen_cauchy1_matrix(int rows, int k, uint8_t *out) {
  memset(out, 0, (size_t)rows * k);
  for (int i = 0; i < k; i++) out[k * i + i] = 1;
  uint8_t *p = out + (size_t)k * k;
  for (int i = k; i < rows; i++)
    for (int j = 0; j < k; j++) *p++ = (uint8_t)orc_gf_inv((uint32_t)((i ^ j) & 0xff), 8);
  return ORC_OK;
}

/* Gauss-Jordan inverse over GF(2^w) (ISA-L gf_invert_matrix for w = 8,
 * jerasure_invert_matrix otherwise; the inverse is unique). */
static int gf_invert(uint32_t *a, uint32_t *inv, int n, int w) {
  for (int i = 0; i < n * n; i++) inv[i] = 0;
  for (int i = 0; i < n; i++) inv[i * n + i] = 1;
  for (int i = 0; i < n; i++) {
    if (a[i * n + i] == 0) {
      int j = i + 1;
      while (j < n && a[j * n + i] == 0) j++;
      if (j == n) return -1;
      for (int c = 0; c < n; c++) {
        uint32_t t = a[i * n + c]; a[i * n + c] = a[j * n + c]; a[j * n + c] = t;
        t = inv[i * n + c]; inv[i * n + c] = inv[j * n + c]; inv[j * n + c] = t;
      }
    }
    uint32_t p = orc_gf_inv(a[i * n + i], w);
    for (int c = 0; c < n; c++) {
      a[i * n + c] = orc_gf_mul(a[i * n + c], p, w);
      inv[i * n + c] = orc_gf_mul(inv[i * n + c], p, w);
    }
    for (int j = 0; j < n; j++) {
      if (j == i) continue;
      uint32_t t = a[j * n + i];
      if (!t) continue;
      for (int c = 0; c < n; c++) {
        inv[j * n + c] ^= orc_gf_mul(t, inv[i * n + c], w);
        a[j * n + c] ^= orc_gf_mul(t, a[i * n + c], w);
      }
    }
  }
  return 0;
}

int orc_isal_invert_matrix(const uint8_t *in, uint8_t *out, int n) {
  uint32_t *a = malloc(sizeof(uint32_t) * n * n), *b = malloc(sizeof(uint32_t) * n * n);
  if (!a || !b) { free(a); free(b); return ORC_E_NOMEM; }
  for (int i = 0; i < n * n; i++) a[i] = in[i];
  int rc = gf_invert(a, b, n, 8);
  if (rc == 0) for (int i = 0; i < n * n; i++) out[i] = (uint8_t)b[i];
  free(a); free(b);
  return rc ? ORC_E_NON_INVERTIBLE : ORC_OK;
}

/* jerasure_invert_bitmatrix: GF(2) Gauss-Jordan (rows of n bytes). */
static int bit_invert(uint8_t *a, uint8_t *inv, int n) {
  memset(inv, 0, (size_t)n * n);
  for (int i = 0; i < n; i++) inv[i * n + i] = 1;
  for (int i = 0; i < n; i++) {
    if (!a[i * n + i]) {
      int j = i + 1;
      while (j < n && !a[j * n + i]) j++;
      if (j == n) return -1;
      for (int c = 0; c < n; c++) {
        uint8_t t = a[i * n + c]; a[i * n + c] = a[j * n + c]; a[j * n + c] = t;
        t = inv[i * n + c]; inv[i * n + c] = inv[j * n + c]; inv[j * n + c] = t;
      }
    }
    for (int j = 0; j < n; j++) {
      if (j != i && a[j * n + i]) {
        for (int c = 0; c < n; c++) { a[j * n + c] ^= a[i * n + c]; inv[j * n + c] ^= inv[i * n + c]; }
      }
    }
  }
  return 0;
}

/* ------------------------------------------------------------------------ */
/* Geometry: roundTo (c_src/common.cpp:24-33) and the block size of every
 * coder (c_src/rscoding.cpp:44, cauchycoding.cpp:49, liberationcoding.cpp:49,
 * irscoding.cpp:46).                                                         */
uint64_t orc_round_to(uint64_t n, uint64_t multiple) {
  if (multiple == 0) return n;
  uint64_t r = n % multiple;
  return r == 0 ? n : n + multiple - r;
}

uint64_t orc_block_size(int k, int w, uint64_t size) {
  uint64_t kw = (uint64_t)k * (uint64_t)w;
  return orc_round_to(orc_round_to(size, kw) / kw, 16) * (uint64_t)w;
}

static int is_prime(int w) { /* c_src/common.cpp:36-47 */
  static const int p55[] = {2,3,5,7,11,13,17,19,23,29,31,37,41,43,47,53,59,61,67,71,
                            73,79,83,89,97,101,103,107,109,113,127,131,137,139,149,151,157,163,167,173,179,
                            181,191,193,197,199,211,223,227,229,233,239,241,251,257};
  for (int i = 0; i < 55; i++)
    if (w % p55[i] == 0) return w == p55[i];
  return 1;
}

/* checkParams of each coder: rscoding.cpp:29-34, cauchycoding.cpp:30-35,
 * liberationcoding.cpp:29-36, irscoding.cpp:32-37; factory nif.cpp:44-72. */
int orc_check_params(int coding, int k, int m, int w) {
  switch (coding) {
    case ORC_VANDRS:
      if (k <= 0 || m <= 0 || w <= 0) return ORC_E_PARAMS;
      if (w != 8 && w != 16 && w != 32) return ORC_E_PARAMS_W_RS;
      if (w == 8 && k + m > 256) return ORC_E_UNSUPPORTED; /* no Vandermonde matrix (NULL) */
      return ORC_OK;
    case ORC_CAUCHYRS:
      if (k <= 0 || m <= 0 || w <= 0) return ORC_E_PARAMS;
      if (w < 31 && (long long)(k + m) > (1ll << w)) return ORC_E_PARAMS_LARGER_W;
      if (w > 32) return ORC_E_UNSUPPORTED;
      return ORC_OK;
    case ORC_LIBERATION:
      if (k <= 0 || m != 2 || w <= 0) return ORC_E_PARAMS_M2;
      if (k > w) return ORC_E_PARAMS_K_LE_W;
      if (w <= 2 || !(w % 2) || !is_prime(w)) return ORC_E_PARAMS_W_PRIME;
      if (w > 32) return ORC_E_UNSUPPORTED;
      return ORC_OK;
    case ORC_ISARS:
      if (k <= 0 || m <= 0 || w <= 0) return ORC_E_PARAMS;
      if (w != 8) return ORC_E_PARAMS_W8;
      if (k + m > 256) return ORC_E_UNSUPPORTED; /* ISA-L matrix rows are bytes */
      return ORC_OK;
    default:
      return ORC_E_INVALID_CODING;
  }
}

/* ------------------------------------------------------------------------ */
/* Region arithmetic: gf-complete region multiply (w = 8: bytes; w = 16/32:
 * little-endian words), as driven by jerasure_matrix_dotprod and ISA-L
 * ec_encode_data.                                                            */
static uint8_t g8mul[256][256];
static pthread_once_t g8once = PTHREAD_ONCE_INIT;
static void g8init(void) {
  for (int a = 0; a < 256; a++)
    for (int b = 0; b < 256; b++) g8mul[a][b] = (uint8_t)orc_gf_mul(a, b, 8);
}

/* dst ^= c * src over `len` bytes */
static void region_madd(int w, uint32_t c, const uint8_t *src, uint8_t *dst, uint64_t len) {
  if (c == 0) return;
  if (w == 8) {
    pthread_once(&g8once, g8init);
    const uint8_t *t = g8mul[c];
    for (uint64_t i = 0; i < len; i++) dst[i] ^= t[src[i]];
    return;
  }
  if (c == 1) { for (uint64_t i = 0; i < len; i++) dst[i] ^= src[i]; return; }
  /* w = 16 / 32: four 256-entry byte-position tables for constant c */
  uint32_t t[4][256];
  for (int p = 0; p < w / 8; p++)
    for (int b = 0; b < 256; b++) t[p][b] = orc_gf_mul(c, (uint32_t)b << (8 * p), w);
  if (w == 16) {
    for (uint64_t i = 0; i + 1 < len; i += 2) {
      uint32_t x = (uint32_t)src[i] | ((uint32_t)src[i + 1] << 8);
      uint32_t y = t[0][x & 0xff] ^ t[1][x >> 8];
      dst[i] ^= (uint8_t)y; dst[i + 1] ^= (uint8_t)(y >> 8);
    }
  } else {
    for (uint64_t i = 0; i + 3 < len; i += 4) {
      uint32_t x = (uint32_t)src[i] | ((uint32_t)src[i + 1] << 8) | ((uint32_t)src[i + 2] << 16) |
                   ((uint32_t)src[i + 3] << 24);
      uint32_t y = t[0][x & 0xff] ^ t[1][(x >> 8) & 0xff] ^ t[2][(x >> 16) & 0xff] ^ t[3][x >> 24];
      dst[i] ^= (uint8_t)y; dst[i + 1] ^= (uint8_t)(y >> 8);
      dst[i + 2] ^= (uint8_t)(y >> 16); dst[i + 3] ^= (uint8_t)(y >> 24);
    }
  }
}

/* jerasure_matrix_dotprod: dst = sum_i row[i] * src_i */
static void dotprod(int w, int n, const uint32_t *row, const uint8_t *const *src, uint8_t *dst,
                    uint64_t len) {
  memset(dst, 0, len);
  for (int i = 0; i < n; i++) region_madd(w, row[i], src[i], dst, len);
}

/* bitmatrix product over packets: out packet (r) = XOR of in packets (c) with
 * B[r][c] = 1.  Packet c of the input = block c / w, bytes [(c%w)*ps, +ps). */
static void bitmatrix_apply(int w, int nin_blocks, int nout_blocks, const uint8_t *B,
                            const uint8_t *const *in, uint8_t *const *out, uint64_t bs) {
  uint64_t ps = bs / (uint64_t)w;
  int cols = nin_blocks * w;
  for (int o = 0; o < nout_blocks; o++)
    for (int r = 0; r < w; r++) {
      uint8_t *dst = out[o] + (uint64_t)r * ps;
      memset(dst, 0, ps);
      const uint8_t *brow = B + (size_t)(o * w + r) * cols;
      for (int c = 0; c < cols; c++)
        if (brow[c]) {
          const uint8_t *s = in[c / w] + (uint64_t)(c % w) * ps;
          for (uint64_t i = 0; i < ps; i++) dst[i] ^= s[i];
        }
    }
}

/* ------------------------------------------------------------------------ */
/* Coding matrices per class */
static int coding_bitmatrix(int coding, int k, int m, int w, uint8_t **B) {
  *B = malloc((size_t)m * w * k * w);
  if (!*B) return ORC_E_NOMEM;
  if (coding == ORC_LIBERATION) return orc_liberation_coding_bitmatrix(k, w, *B);
  uint32_t *mat = malloc(sizeof(uint32_t) * m * k);
  if (!mat) return ORC_E_NOMEM;
  int rc = orc_cauchy_good_general_coding_matrix(k, m, w, mat);
  if (!rc) rc = orc_matrix_to_bitmatrix(k, m, w, mat, *B);
  free(mat);
  return rc;
}

static int coding_matrix(int coding, int k, int m, int w, uint32_t *mat) {
  if (coding == ORC_VANDRS) return orc_vandermonde_coding_matrix(k, m, w, mat);
  /* isars */
  uint8_t *a = malloc((size_t)(k + m) * k);
  if (!a) return ORC_E_NOMEM;
  orc_isal_gen_cauchy1_matrix(k + m, k, a);
  for (int i = 0; i < m * k; i++) mat[i] = a[(size_t)k * k + i];
  free(a);
  return ORC_OK;
}

/* RSCoding::doEncode (rscoding.cpp:36-85) / CauchyCoding::doEncode
 * (cauchycoding.cpp:37-89) / LiberationCoding::doEncode (liberationcoding.cpp:38-85)
 * / IRSCoding::doEncode (irscoding.cpp:39-84).  The returned block list is
 * id-ordered: block i = bytes [i*bs,(i+1)*bs) of the zero-padded object, then
 * the m coding blocks. */
int orc_encode(int coding, int k, int m, int w, const uint8_t *obj, uint64_t size,
               uint8_t *blocks) {
  int rc = orc_check_params(coding, k, m, w);
  if (rc) return rc;
  uint64_t bs = orc_block_size(k, w, size);
  memset(blocks, 0, (size_t)(k + m) * bs);
  if (size) memcpy(blocks, obj, size);
  if (bs == 0) return ORC_OK;
  const uint8_t *data[256];
  uint8_t *code[256];
  if (k > 256 || m > 256) return ORC_E_UNSUPPORTED;
  for (int j = 0; j < k; j++) data[j] = blocks + (uint64_t)j * bs;
  for (int i = 0; i < m; i++) code[i] = blocks + (uint64_t)(k + i) * bs;
  if (coding == ORC_VANDRS || coding == ORC_ISARS) {
    uint32_t *mat = malloc(sizeof(uint32_t) * m * k);
    if (!mat) return ORC_E_NOMEM;
    rc = coding_matrix(coding, k, m, w, mat);
    if (!rc)
      for (int i = 0; i < m; i++) dotprod(w, k, mat + (size_t)i * k, data, code[i], bs);
    free(mat);
    return rc;
  }
  uint8_t *B;
  rc = coding_bitmatrix(coding, k, m, w, &B);
  if (!rc) bitmatrix_apply(w, k, m, B, data, code, bs);
  free(B);
  return rc;
}

/* Shared validation of doDecode/doRepair (e.g. rscoding.cpp:89-104). */
static int validate_blocks(int k, int m, const int *ids, int n, int present[]) {
  for (int i = 0; i < k + m; i++) present[i] = -1;
  int uniq = 0;
  for (int i = 0; i < n; i++) {
    if (ids[i] < 0 || ids[i] >= k + m) return ORC_E_BAD_ID;
    if (present[ids[i]] < 0) uniq++;
    present[ids[i]] = i; /* the last listed block of an id wins, as in blocks[blockId] */
  }
  if (uniq < k) return ORC_E_NOT_ENOUGH;
  if (uniq < n) return ORC_E_NOT_UNIQUE;
  return ORC_OK;
}

/* Linear map from survivors to wanted block ids.
 *  - vandrs / cauchyrs / liberation: survivors = first k non-erased ids in
 *    ascending order (jerasure_make_decoding_matrix dm_ids;
 *    set_up_ids_for_scheduled_decoding).
 *  - isars: survivors = the first k listed blocks (IRSCoding::gf_gen_decode_matrix,
 *    irscoding.cpp:188-220).
 * Computes, for GF(2^w) codes, rows[nwant][k] (out = rows * survivors), and
 * for bitmatrix codes, brows[nwant*w][k*w].                                  */
static int decode_map_gf(int coding, int k, int m, int w, const uint32_t *C, const int *surv,
                         const int *want, int nwant, uint32_t *rows) {
  uint32_t *G = malloc(sizeof(uint32_t) * k * k), *inv = malloc(sizeof(uint32_t) * k * k);
  if (!G || !inv) { free(G); free(inv); return ORC_E_NOMEM; }
  for (int i = 0; i < k; i++)
    for (int j = 0; j < k; j++)
      G[i * k + j] = surv[i] < k ? (uint32_t)(surv[i] == j) : C[(surv[i] - k) * k + j];
  if (gf_invert(G, inv, k, w)) { free(G); free(inv); return ORC_E_NON_INVERTIBLE; }
  for (int o = 0; o < nwant; o++) {
    if (want[o] < k) {
      memcpy(rows + (size_t)o * k, inv + (size_t)want[o] * k, sizeof(uint32_t) * k);
    } else {
      const uint32_t *c = C + (size_t)(want[o] - k) * k;
      for (int j = 0; j < k; j++) {
        uint32_t s = 0;
        for (int l = 0; l < k; l++) s ^= orc_gf_mul(c[l], inv[l * k + j], w);
        rows[(size_t)o * k + j] = s;
      }
    }
  }
  free(G); free(inv);
  return ORC_OK;
}

static int decode_map_bit(int k, int m, int w, const uint8_t *B, const int *surv, const int *want,
                          int nwant, uint8_t *brows) {
  int n = k * w;
  uint8_t *G = malloc((size_t)n * n), *inv = malloc((size_t)n * n);
  if (!G || !inv) { free(G); free(inv); return ORC_E_NOMEM; }
  for (int i = 0; i < k; i++)
    for (int r = 0; r < w; r++) {
      uint8_t *g = G + (size_t)(i * w + r) * n;
      if (surv[i] < k) { memset(g, 0, n); g[surv[i] * w + r] = 1; }
      else memcpy(g, B + (size_t)((surv[i] - k) * w + r) * n, n);
    }
  if (bit_invert(G, inv, n)) { free(G); free(inv); return ORC_E_NON_INVERTIBLE; }
  for (int o = 0; o < nwant; o++)
    for (int r = 0; r < w; r++) {
      uint8_t *dst = brows + (size_t)(o * w + r) * n;
      if (want[o] < k) {
        memcpy(dst, inv + (size_t)(want[o] * w + r) * n, n);
      } else {
        const uint8_t *b = B + (size_t)((want[o] - k) * w + r) * n;
        memset(dst, 0, n);
        for (int l = 0; l < n; l++)
          if (b[l]) for (int c = 0; c < n; c++) dst[c] ^= inv[(size_t)l * n + c];
      }
    }
  free(G); free(inv);
  return ORC_OK;
}

/* Produce the blocks `want` (any ids) from the listed blocks. out[o] = bs bytes. */
static int reconstruct(int coding, int k, int m, int w, const uint8_t *const *blocks,
                       const int *ids, int n, const int present[], uint64_t bs, const int *want,
                       int nwant, uint8_t *const *out) {
  int surv[256];
  if (coding == ORC_ISARS) {
    for (int i = 0; i < k; i++) surv[i] = ids[i];
  } else {
    int j = 0;
    for (int i = 0; i < k + m && j < k; i++)
      if (present[i] >= 0) surv[j++] = i;
  }
  const uint8_t *sv[256];
  for (int i = 0; i < k; i++) sv[i] = blocks[present[surv[i]]];
  if (coding == ORC_ISARS) for (int i = 0; i < k; i++) sv[i] = blocks[i];
  int rc;
  if (coding == ORC_VANDRS || coding == ORC_ISARS) {
    uint32_t *C = malloc(sizeof(uint32_t) * m * k), *rows = malloc(sizeof(uint32_t) * nwant * k);
    if (!C || !rows) { free(C); free(rows); return ORC_E_NOMEM; }
    rc = coding_matrix(coding, k, m, w, C);
    if (!rc) rc = decode_map_gf(coding, k, m, w, C, surv, want, nwant, rows);
    if (!rc)
      for (int o = 0; o < nwant; o++) dotprod(w, k, rows + (size_t)o * k, sv, out[o], bs);
    free(C); free(rows);
    return rc;
  }
  if (bs % (uint64_t)w) return ORC_E_BAD_SIZE;
  uint8_t *B, *brows = malloc((size_t)nwant * w * k * w);
  if (!brows) return ORC_E_NOMEM;
  rc = coding_bitmatrix(coding, k, m, w, &B);
  if (!rc) rc = decode_map_bit(k, m, w, B, surv, want, nwant, brows);
  if (!rc) bitmatrix_apply(w, k, nwant, brows, sv, out, bs);
  free(B); free(brows);
  return rc;
}

/* doDecode of each coder (rscoding.cpp:87-154 etc.): output = first `size`
 * bytes of D0..D(k-1).  (The reference's fast path overflows its buffer when
 * trailing data blocks are pure padding, rscoding.cpp:116-120; the intended
 * semantics are restated here.) */
int orc_decode(int coding, int k, int m, int w, const uint8_t *const *blocks, const int *ids,
               int n, uint64_t bs, uint64_t size, uint8_t *out) {
  int rc = orc_check_params(coding, k, m, w);
  if (rc) return rc;
  if (k + m > 256) return ORC_E_UNSUPPORTED;
  int present[256];
  rc = validate_blocks(k, m, ids, n, present);
  if (rc) return rc;
  if (size > (uint64_t)k * bs) return ORC_E_BAD_SIZE;
  int want[256], nwant = 0;
  for (int i = 0; i < k; i++)
    if (present[i] < 0) want[nwant++] = i;
  uint8_t *rec = NULL;
  uint8_t *outp[256];
  if (nwant) {
    rec = malloc((size_t)nwant * bs + 1);
    if (!rec) return ORC_E_NOMEM;
    for (int o = 0; o < nwant; o++) outp[o] = rec + (uint64_t)o * bs;
    rc = reconstruct(coding, k, m, w, blocks, ids, n, present, bs, want, nwant, outp);
    if (rc) { free(rec); return rc; }
  }
  int o = 0;
  for (int i = 0; i < k; i++) {
    uint64_t off = (uint64_t)i * bs;
    if (off >= size) break;
    uint64_t len = size - off < bs ? size - off : bs;
    const uint8_t *src = present[i] >= 0 ? blocks[present[i]] : outp[o];
    memcpy(out + off, src, len);
    if (present[i] < 0) o++;
  }
  free(rec);
  return ORC_OK;
}

/* doRepair of each coder (rscoding.cpp:156-211, cauchycoding.cpp:159-213,
 * liberationcoding.cpp:156-208, irscoding.cpp:146-186). */
int orc_repair(int coding, int k, int m, int w, const uint8_t *const *blocks, const int *ids,
               int n, uint64_t bs, const int *rep, int nrep, uint8_t *out) {
  int rc = orc_check_params(coding, k, m, w);
  if (rc) return rc;
  if (k + m > 256 || nrep > 256) return ORC_E_UNSUPPORTED;
  int present[256];
  rc = validate_blocks(k, m, ids, n, present);
  if (rc) return rc;
  int want[256], nwant = 0;
  uint8_t *outp[256];
  for (int r = 0; r < nrep; r++) {
    if (rep[r] < 0 || rep[r] >= k + m) return ORC_E_BAD_ID;
    /* jerasure classes return a listed block as-is; isars recomputes it */
    if (coding != ORC_ISARS && present[rep[r]] >= 0) {
      memcpy(out + (uint64_t)r * bs, blocks[present[rep[r]]], bs);
    } else {
      outp[nwant] = out + (uint64_t)r * bs;
      want[nwant++] = rep[r];
    }
  }
  if (nwant) rc = reconstruct(coding, k, m, w, blocks, ids, n, present, bs, want, nwant, outp);
  return rc;
}

/* ------------------------------------------------------------------------ */
/* CPU baseline: vandrs(k,m,8) with ISA-L's split-nibble table technique
 * (ec_init_tables: 32 B per coefficient; ec_encode_data: PSHUFB lookups),
 * multi-threaded across independent objects.                                */
int orc_simd_level(void) {
#if defined(__x86_64__)
  __builtin_cpu_init();
  if (__builtin_cpu_supports("avx512f") && __builtin_cpu_supports("avx512bw") &&
      __builtin_cpu_supports("gfni"))
    return 3;
  if (__builtin_cpu_supports("avx2")) return 2;
#endif
  return 0;
}

/* ISA-L's AVX-512 + GFNI technique (ec_encode_data_avx512_gfni): multiply by
 * c is an 8x8 GF(2) matrix applied to every byte by vgf2p8affineqb; row i of
 * the matrix (output bit i) is byte 7-i of the qword. */
static uint64_t gfni_matrix(uint32_t c) {
  pthread_once(&g8once, g8init);
  uint64_t A = 0;
  for (int i = 0; i < 8; i++) {
    uint64_t row = 0;
    for (int j = 0; j < 8; j++)
      if ((g8mul[c][1 << j] >> i) & 1) row |= 1ull << j;
    A |= row << (8 * (7 - i));
  }
  return A;
}

static void init_tables(int nrow, int ncol, const uint32_t *rows, uint8_t *tbl) {
  pthread_once(&g8once, g8init);
  for (int r = 0; r < nrow; r++)
    for (int j = 0; j < ncol; j++) {
      uint8_t *t = tbl + ((size_t)r * ncol + j) * 32;
      uint32_t c = rows[r * ncol + j];
      for (int x = 0; x < 16; x++) { t[x] = g8mul[c][x]; t[16 + x] = g8mul[c][x << 4]; }
    }
}

static void apply_scalar(int nin, int nout, const uint8_t *tbl, const uint8_t *const *in,
                         uint8_t *const *out, uint64_t len) {
  for (int o = 0; o < nout; o++) {
    memset(out[o], 0, len);
    for (int j = 0; j < nin; j++) {
      const uint8_t *t = tbl + ((size_t)o * nin + j) * 32;
      const uint8_t *s = in[j];
      uint8_t *d = out[o];
      for (uint64_t i = 0; i < len; i++) d[i] ^= t[s[i] & 15] ^ t[16 + (s[i] >> 4)];
    }
  }
}

#if defined(__x86_64__)
__attribute__((target("avx2"))) static void apply_avx2(int nin, int nout, const uint8_t *tbl,
                                                        const uint8_t *const *in,
                                                        uint8_t *const *out, uint64_t len) {
  const __m256i mask = _mm256_set1_epi8(0x0f);
  uint64_t i = 0;
  for (; i + 32 <= len; i += 32) {
    __m256i acc[16];
    for (int o = 0; o < nout; o++) acc[o] = _mm256_setzero_si256();
    for (int j = 0; j < nin; j++) {
      __m256i x = _mm256_loadu_si256((const __m256i *)(in[j] + i));
      __m256i lo = _mm256_and_si256(x, mask);
      __m256i hi = _mm256_and_si256(_mm256_srli_epi64(x, 4), mask);
      for (int o = 0; o < nout; o++) {
        const uint8_t *t = tbl + ((size_t)o * nin + j) * 32;
        __m256i tl = _mm256_broadcastsi128_si256(_mm_loadu_si128((const __m128i *)t));
        __m256i th = _mm256_broadcastsi128_si256(_mm_loadu_si128((const __m128i *)(t + 16)));
        acc[o] = _mm256_xor_si256(acc[o], _mm256_xor_si256(_mm256_shuffle_epi8(tl, lo),
                                                           _mm256_shuffle_epi8(th, hi)));
      }
    }
    for (int o = 0; o < nout; o++) _mm256_storeu_si256((__m256i *)(out[o] + i), acc[o]);
  }
  if (i < len) {
    const uint8_t *in2[256];
    uint8_t *out2[256];
    for (int j = 0; j < nin; j++) in2[j] = in[j] + i;
    for (int o = 0; o < nout; o++) out2[o] = out[o] + i;
    apply_scalar(nin, nout, tbl, in2, out2, len - i);
  }
}
#endif

#if defined(__x86_64__)
/* ISA-L's gf_Nvect_dot_prod_avx512_gfni shape for N = nout <= 4 output rows:
 * the row count compiled in (NOUT is a literal at every call site of this
 * always-inline body), so the accumulators live in zmm registers, not in a
 * run-time-indexed array on the stack; two 64-byte vectors per iteration (two
 * independent XOR chains per row); each coefficient's affine matrix is a
 * broadcast memory operand of vgf2p8affineqb.  Returns the bytes done (a
 * multiple of 128; the caller finishes the rest). */
__attribute__((target("avx512f,avx512bw,gfni"), always_inline)) static inline uint64_t
gfni_rows(int nin, const int NOUT, const uint64_t *mats, const uint8_t *const *in,
          uint8_t *const *out, uint64_t len) {
  uint64_t i = 0;
  for (; i + 128 <= len; i += 128) {
    __m512i a0 = _mm512_setzero_si512(), a1 = a0, a2 = a0, a3 = a0;
    __m512i b0 = a0, b1 = a0, b2 = a0, b3 = a0;
    for (int j = 0; j < nin; j++) {
      const __m512i x = _mm512_loadu_si512((const void *)(in[j] + i));
      const __m512i y = _mm512_loadu_si512((const void *)(in[j] + i + 64));
      const uint64_t *mj = mats + j;
#define GF_ROW(o, A, B)                                                          \
      if (NOUT > o) {                                                            \
        const __m512i M = _mm512_set1_epi64((long long)mj[(size_t)(o) * nin]);   \
        A = _mm512_xor_si512(A, _mm512_gf2p8affine_epi64_epi8(x, M, 0));         \
        B = _mm512_xor_si512(B, _mm512_gf2p8affine_epi64_epi8(y, M, 0));         \
      }
      GF_ROW(0, a0, b0)
      GF_ROW(1, a1, b1)
      GF_ROW(2, a2, b2)
      GF_ROW(3, a3, b3)
#undef GF_ROW
    }
    _mm512_storeu_si512((void *)(out[0] + i), a0);
    _mm512_storeu_si512((void *)(out[0] + i + 64), b0);
    if (NOUT > 1) {
      _mm512_storeu_si512((void *)(out[1] + i), a1);
      _mm512_storeu_si512((void *)(out[1] + i + 64), b1);
    }
    if (NOUT > 2) {
      _mm512_storeu_si512((void *)(out[2] + i), a2);
      _mm512_storeu_si512((void *)(out[2] + i + 64), b2);
    }
    if (NOUT > 3) {
      _mm512_storeu_si512((void *)(out[3] + i), a3);
      _mm512_storeu_si512((void *)(out[3] + i + 64), b3);
    }
  }
  return i;
}

__attribute__((target("avx512f,avx512bw,gfni"))) static void apply_gfni(
    int nin, int nout, const uint64_t *mats, const uint8_t *tbl, const uint8_t *const *in,
    uint8_t *const *out, uint64_t len) {
  uint64_t i = 0;
  /* the rows in groups of at most 4, each group one specialised pass (ISA-L
   * runs m > 6 rows as several passes the same way) */
  if (nout <= 16) {
    uint64_t done = len;
    for (int o0 = 0; o0 < nout; o0 += 4) {
      const int n = nout - o0 < 4 ? nout - o0 : 4;
      const uint64_t *mo = mats + (size_t)o0 * nin;
      uint8_t *const *oo = out + o0;
      const uint64_t d = n == 4   ? gfni_rows(nin, 4, mo, in, oo, len)
                         : n == 3 ? gfni_rows(nin, 3, mo, in, oo, len)
                         : n == 2 ? gfni_rows(nin, 2, mo, in, oo, len)
                                  : gfni_rows(nin, 1, mo, in, oo, len);
      done = d;
    }
    i = nout > 0 ? done : len;
  }
  for (; i + 64 <= len; i += 64) {
    __m512i acc[16];
    for (int o = 0; o < nout; o++) acc[o] = _mm512_setzero_si512();
    for (int j = 0; j < nin; j++) {
      const __m512i x = _mm512_loadu_si512((const void *)(in[j] + i));
      for (int o = 0; o < nout; o++)
        acc[o] = _mm512_xor_si512(
            acc[o], _mm512_gf2p8affine_epi64_epi8(x, _mm512_set1_epi64((long long)mats[o * nin + j]), 0));
    }
    for (int o = 0; o < nout; o++) _mm512_storeu_si512((void *)(out[o] + i), acc[o]);
  }
  if (i < len) {
    const uint8_t *in2[256];
    uint8_t *out2[256];
    for (int j = 0; j < nin; j++) in2[j] = in[j] + i;
    for (int o = 0; o < nout; o++) out2[o] = out[o] + i;
    apply_scalar(nin, nout, tbl, in2, out2, len - i);
  }
}
#endif

typedef struct {
  int op, k, m, nout, simd;
  const uint8_t *objs;
  uint64_t stride, size, bs;
  int o0, o1;
  uint8_t *parity;
  const uint8_t *tbl;
  const uint64_t *mats; /* GFNI affine matrices, nout x k */
  const int *want;      /* decode: erased data ids */
  const int *surv;      /* decode: survivor ids */
  const uint32_t *coef; /* nout x k coefficients (structure 1: ones are copies / xors) */
  int structure;        /* 0: one pass over all rows (ISA-L ec_encode_data);
                           1: Jerasure's per-(row, input) region passes;
                           2: the one pass with scalar table lookups */
} bench_job;

/* Jerasure's structure (jerasure_matrix_encode -> jerasure_matrix_dotprod per
 * coding row, rscoding.cpp:71; jerasure_matrix_decode_data per erased row,
 * rscoding.cpp:147): for each output row, first the inputs whose coefficient
 * is 1 (memcpy for the first, galois_region_xor after), then one
 * galois_w08_region_multiply pass per other nonzero coefficient, each over
 * the whole block, accumulating into the destination from the second pass
 * on (read-modify-write).  The multiply is gf-complete's w = 8 split-table
 * technique (two 16-entry nibble tables and PSHUFB), here 32 B wide. */
static void region_mul_scalar(const uint8_t *t, const uint8_t *s, uint8_t *d, uint64_t len,
                              int add) {
  if (add)
    for (uint64_t i = 0; i < len; i++) d[i] ^= t[s[i] & 15] ^ t[16 + (s[i] >> 4)];
  else
    for (uint64_t i = 0; i < len; i++) d[i] = t[s[i] & 15] ^ t[16 + (s[i] >> 4)];
}

static void region_xor(const uint8_t *s, uint8_t *d, uint64_t len) {
  uint64_t i = 0;
  for (; i + 8 <= len; i += 8) {
    uint64_t a, b;
    memcpy(&a, s + i, 8);
    memcpy(&b, d + i, 8);
    a ^= b;
    memcpy(d + i, &a, 8);
  }
  for (; i < len; i++) d[i] ^= s[i];
}

#if defined(__x86_64__)
__attribute__((target("avx2"))) static void region_mul_avx2(const uint8_t *t, const uint8_t *s,
                                                            uint8_t *d, uint64_t len, int add) {
  const __m256i mask = _mm256_set1_epi8(0x0f);
  const __m256i tl = _mm256_broadcastsi128_si256(_mm_loadu_si128((const __m128i *)t));
  const __m256i th = _mm256_broadcastsi128_si256(_mm_loadu_si128((const __m128i *)(t + 16)));
  uint64_t i = 0;
  for (; i + 32 <= len; i += 32) {
    const __m256i x = _mm256_loadu_si256((const __m256i *)(s + i));
    __m256i r = _mm256_xor_si256(_mm256_shuffle_epi8(tl, _mm256_and_si256(x, mask)),
                                 _mm256_shuffle_epi8(th, _mm256_and_si256(_mm256_srli_epi64(x, 4), mask)));
    if (add) r = _mm256_xor_si256(r, _mm256_loadu_si256((const __m256i *)(d + i)));
    _mm256_storeu_si256((__m256i *)(d + i), r);
  }
  if (i < len) region_mul_scalar(t, s + i, d + i, len - i, add);
}
#endif

static void apply_regions(int nin, int nout, const uint32_t *coef, const uint8_t *tbl, int simd,
                          const uint8_t *const *in, uint8_t *const *out, uint64_t len) {
  for (int o = 0; o < nout; o++) {
    int init = 0;
    for (int j = 0; j < nin; j++) {
      if (coef[o * nin + j] != 1) continue;
      if (init) region_xor(in[j], out[o], len);
      else memcpy(out[o], in[j], len);
      init = 1;
    }
    for (int j = 0; j < nin; j++) {
      const uint32_t c = coef[o * nin + j];
      if (c <= 1) continue;
      const uint8_t *t = tbl + ((size_t)o * nin + j) * 32;
#if defined(__x86_64__)
      if (simd >= 2) region_mul_avx2(t, in[j], out[o], len, init);
      else
#endif
        region_mul_scalar(t, in[j], out[o], len, init);
      init = 1;
    }
    if (!init) memset(out[o], 0, len);
  }
}

/* One object of a bench job: RSCoding::doEncode's stripe staging, then the
 * encode, or the in-place decode of the job's erased data blocks.  `tail` is
 * a k*bs scratch buffer. */
static void bench_object_at(const bench_job *J, const uint8_t *obj, uint8_t *par, uint8_t *tail) {
  uint64_t bs = J->bs;
  int k = J->k, m = J->m;
  {
    /* stripe staging exactly as RSCoding::doEncode: whole blocks alias the
     * object, the tail block is copied into a zeroed buffer */
    const uint8_t *blk[256];
    uint64_t filled = bs ? J->size / bs : 0;
    if (filled > (uint64_t)k) filled = k;
    memset(tail, 0, (k - filled) * bs);
    memcpy(tail, obj + filled * bs, J->size - filled * bs);
    for (int j = 0; j < k; j++)
      blk[j] = (uint64_t)j < filled ? obj + (uint64_t)j * bs : tail + (j - filled) * bs;
    const uint8_t *in[256];
    uint8_t *out[256];
    int nin;
    if (J->op == 0) {
      nin = k;
      for (int j = 0; j < k; j++) in[j] = blk[j];
      for (int i = 0; i < m; i++) out[i] = par + (uint64_t)i * bs;
    } else {
      nin = k;
      for (int j = 0; j < k; j++) in[j] = J->surv[j] < k ? blk[J->surv[j]] : par + (uint64_t)(J->surv[j] - k) * bs;
      /* in place, as the GPU decode: the rebuilt data blocks overwrite their
       * own (identical) bytes in the object / staged tail */
      for (int i = 0; i < J->nout; i++) out[i] = (uint8_t *)blk[J->want[i]];
    }
    if (J->structure == 1) apply_regions(nin, J->nout, J->coef, J->tbl, J->simd, in, out, bs);
    else if (J->structure == 2) apply_scalar(nin, J->nout, J->tbl, in, out, bs);
    else
#if defined(__x86_64__)
    if (J->simd >= 3) apply_gfni(nin, J->nout, J->mats, J->tbl, in, out, bs);
    else if (J->simd >= 2) apply_avx2(nin, J->nout, J->tbl, in, out, bs);
    else
#endif
      apply_scalar(nin, J->nout, J->tbl, in, out, bs);
    /* decode in place: a rebuilt block staged in the tail buffer goes back
     * into the object (its valid bytes) */
    if (J->op != 0)
      for (int i = 0; i < J->nout; i++) {
        uint64_t b = (uint64_t)J->want[i];
        if (b >= filled && b * bs < J->size) {
          uint64_t n = J->size - b * bs < bs ? J->size - b * bs : bs;
          memcpy((uint8_t *)obj + b * bs, out[i], n);
        }
      }
  }
}

static void bench_object(const bench_job *J, int o, uint8_t *tail) {
  bench_object_at(J, J->objs + (uint64_t)o * J->stride,
                  J->parity + (uint64_t)o * J->m * J->bs, tail);
}

static void *bench_worker(void *arg) {
  bench_job *J = arg;
  uint8_t *tail = aligned_alloc(64, orc_round_to(J->bs * (uint64_t)J->k + 64, 64));
  for (int o = J->o0; o < J->o1; o++) bench_object(J, o, tail);
  free(tail);
  return NULL;
}

/* The coefficient tables of one bench op: encode, or the decode of the
 * erased data blocks from the first k intact ids. */
typedef struct {
  int nout, surv[256], want[256];
  uint8_t *tbl;   /* (m+k) x k x 32 split tables */
  uint64_t *mats; /* nout x k GFNI matrices */
  uint32_t *coef; /* nout x k coefficients */
} bench_plan;

static int bench_plan_make(bench_plan *P, int op, int k, int m, const int *erased, int nerased) {
  uint32_t *C = malloc(sizeof(uint32_t) * m * k);
  uint32_t *rows = malloc(sizeof(uint32_t) * (m + k) * k);
  P->tbl = malloc((size_t)(m + k) * k * 32);
  P->mats = NULL;
  P->coef = NULL;
  int *surv = P->surv, *want = P->want, nout = 0;
  int rc = orc_vandermonde_coding_matrix(k, m, 8, C);
  if (rc) goto done;
  if (op == 0) {
    nout = m;
    memcpy(rows, C, sizeof(uint32_t) * m * k);
  } else {
    /* erased ids may include coding blocks: they are only excluded from the
     * survivors; the rebuilt (wanted) blocks are the erased data blocks */
    int er[256] = {0};
    for (int i = 0; i < nerased; i++) {
      if (erased[i] < 0 || erased[i] >= k + m) { rc = ORC_E_PARAMS; goto done; }
      er[erased[i]] = 1;
    }
    int j = 0;
    for (int i = 0; i < k + m && j < k; i++) if (!er[i]) surv[j++] = i;
    if (j < k) { rc = ORC_E_PARAMS; goto done; }
    nout = 0;
    for (int i = 0; i < k; i++) if (er[i]) want[nout++] = i;
    rc = decode_map_gf(ORC_VANDRS, k, m, 8, C, surv, want, nout, rows);
    if (rc) goto done;
  }
  P->nout = nout;
  init_tables(nout, k, rows, P->tbl);
  P->mats = malloc(sizeof(uint64_t) * (size_t)(nout ? nout : 1) * k);
  for (int i = 0; i < nout * k; i++) P->mats[i] = gfni_matrix(rows[i]);
  P->coef = rows;
  rows = NULL;
done:
  free(C);
  free(rows);
  if (rc) { free(P->tbl); P->tbl = NULL; }
  return rc;
}

static void bench_plan_free(bench_plan *P) {
  free(P->tbl);
  free(P->mats);
  free(P->coef);
}

int orc_bench_rs8(int op, int k, int m, const uint8_t *objs, uint64_t obj_stride, uint64_t size,
                  int nobj, uint8_t *parity, const int *erased, int nerased, int threads,
                  int force_scalar) {
  if (k <= 0 || m <= 0 || k + m > 256 || threads <= 0 || nerased > m) return ORC_E_PARAMS;
  uint64_t bs = orc_block_size(k, 8, size);
  bench_plan P;
  int rc = bench_plan_make(&P, op, k, m, erased, nerased);
  if (rc) return rc;
  int nout = P.nout;
  const uint8_t *tbl = P.tbl;
  const uint64_t *mats = P.mats;
  const int *want = P.want, *surv = P.surv;
  {
    pthread_t th[256];
    bench_job jobs[256];
    if (threads > 256) threads = 256;
    int simd = force_scalar ? 0 : orc_simd_level();
    if (force_scalar > 1) simd = force_scalar;  /* 2: force avx2, 3: force gfni */
    for (int t = 0; t < threads; t++) {
      bench_job *J = &jobs[t];
      J->op = op; J->k = k; J->m = m; J->nout = nout; J->simd = simd;
      J->objs = objs; J->stride = obj_stride; J->size = size; J->bs = bs;
      J->o0 = (int)((long long)nobj * t / threads);
      J->o1 = (int)((long long)nobj * (t + 1) / threads);
      J->parity = parity; J->tbl = tbl; J->mats = mats; J->want = want; J->surv = surv;
      J->coef = P.coef; J->structure = 0;
      pthread_create(&th[t], NULL, bench_worker, J);
    }
    for (int t = 0; t < threads; t++) pthread_join(th[t], NULL);
  }
  bench_plan_free(&P);
  return 0;
}

/* The timed CPU baseline (bench.py cpu_baseline): `threads` workers, worker
 * t pinned to cpus[t], each copying ITS slice of the sample (objects
 * [o0, o1) of src) into buffers it allocates and touches itself, so every
 * page lives on the worker's own NUMA node; then passes of >= pass_s
 * seconds, each a whole number of rounds of (encode every object, then
 * decode data blocks `erased` in place) by all workers between two barriers,
 * until total_s seconds and min_passes passes have run.  rates[i] = GiB/s of
 * object payload (2 x objects x size per round) of pass i; returns the number
 * of passes (<= max_passes) or a negative ORC_E_*.  parity_out (nobj x m x
 * bs) receives the workers' encode of the sample, for the parity check.
 * structure 0: ISA-L's one pass per object (apply_gfni / apply_avx2);
 * structure 2: the same pass with scalar split-table lookups (apply_scalar);
 * structure 1: Jerasure's per-(row, input) region passes (apply_regions).
 * throttled_s (nullable, max_passes): the cgroup's CFS-throttled seconds
 * during each pass, -1 where cpu.stat is unreadable.  warm_s > 0: untimed
 * warm-up passes first (see below), their rates in warm_rates[0..*nwarm). */
/* Objects are handed out from a shared counter per phase (chunks of
 * kBenchChunk), not as fixed slices: a worker whose core another tenant of
 * the host takes for a while does fewer objects instead of holding every
 * other worker at the round's barrier. */
enum { kBenchChunk = 2 };

typedef struct {
  const uint8_t **obj;  /* per object of the sample: its first-touched copy */
  uint8_t **par;        /* and its parity rows */
  int nobj;
  volatile int next[2]; /* per phase (0 encode, 1 decode): next object to hand out */
  pthread_barrier_t mid; /* workers only: every encode done before any decode */
} bench_queue;

typedef struct {
  const uint8_t *src;
  uint64_t src_stride;
  int cpu;
  bench_job enc, dec;
  uint8_t *objs, *par, *tail;
  pthread_barrier_t *start, *done;
  volatile int *stop;
  bench_queue *q;
  int o0;               /* first object of this worker's first-touched slice */
  int err, pinned;
} pinned_worker;

static void bench_phase(const bench_job *J, bench_queue *q, int ph, uint8_t *tail) {
  for (;;) {
    const int o = __atomic_fetch_add(&q->next[ph], kBenchChunk, __ATOMIC_RELAXED);
    if (o >= q->nobj) return;
    const int e = o + kBenchChunk < q->nobj ? o + kBenchChunk : q->nobj;
    for (int i = o; i < e; i++)
      if (q->obj[i]) bench_object_at(J, q->obj[i], q->par[i], tail);  /* NULL: its worker failed */
  }
}

static void *pinned_main(void *arg) {
  pinned_worker *W = arg;
#if defined(__linux__)
  if (W->cpu >= 0) {  /* best effort: a refused pin leaves the worker unpinned */
    cpu_set_t set;
    CPU_ZERO(&set);
    CPU_SET(W->cpu, &set);
    W->pinned = pthread_setaffinity_np(pthread_self(), sizeof(set), &set) == 0;
  }
#endif
  const int n = W->enc.o1 - W->enc.o0;
  const uint64_t size = W->enc.size, bs = W->enc.bs;
  const int k = W->enc.k, m = W->enc.m;
  W->objs = aligned_alloc(64, orc_round_to((uint64_t)(n ? n : 1) * size + 64, 64));
  W->par = aligned_alloc(64, orc_round_to((uint64_t)(n ? n : 1) * m * bs + 64, 64));
  W->tail = aligned_alloc(64, orc_round_to(bs * (uint64_t)k + 64, 64));
  if (!W->objs || !W->par || !W->tail) W->err = 1;
  else {
    for (int o = 0; o < n; o++)  /* first touch, by this pinned thread */
      memcpy(W->objs + (uint64_t)o * size, W->src + (uint64_t)(W->enc.o0 + o) * W->src_stride, size);
    memset(W->par, 0, (uint64_t)n * m * bs);
    memset(W->tail, 0, bs * (uint64_t)k);
  }
  W->enc.objs = W->dec.objs = W->objs;
  W->enc.stride = W->dec.stride = size;
  W->enc.parity = W->dec.parity = W->par;
  W->enc.o1 = W->dec.o1 = n;
  W->enc.o0 = W->dec.o0 = 0;
  if (!W->err)
    for (int o = 0; o < n; o++) {
      W->q->obj[W->o0 + o] = W->objs + (uint64_t)o * size;
      W->q->par[W->o0 + o] = W->par + (uint64_t)o * m * bs;
    }
  for (;;) {
    pthread_barrier_wait(W->start);
    if (*W->stop) break;
    /* (a failed allocation anywhere stops the run: the main thread checks
     * every worker's err before the first timed round) */
    bench_phase(&W->enc, W->q, 0, W->tail);
    pthread_barrier_wait(&W->q->mid);
    bench_phase(&W->dec, W->q, 1, W->tail);
    pthread_barrier_wait(W->done);
  }
  return NULL;
}

static double now_s(void) {
  struct timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return (double)ts.tv_sec + 1e-9 * (double)ts.tv_nsec;
}

/* The cgroup's cumulative CFS-throttled time in microseconds (cpu.stat
 * throttled_usec), or -1 where unreadable. */
static long long cgroup_throttled_us(void) {
  FILE *f = fopen("/sys/fs/cgroup/cpu.stat", "r");
  if (!f) return -1;
  char key[64];
  long long v, r = -1;
  while (fscanf(f, "%63s %lld", key, &v) == 2)
    if (!strcmp(key, "throttled_usec")) { r = v; break; }
  fclose(f);
  return r;
}

int orc_bench_rs8_pinned(int k, int m, const uint8_t *src, uint64_t src_stride, uint64_t size,
                         int nobj, const int *erased, int nerased, int threads, const int *cpus,
                         double pass_s, double total_s, int min_passes, double *rates,
                         int max_passes, uint8_t *parity_out, int structure,
                         double *throttled_s, double warm_s, double *warm_rates, int max_warm,
                         int *nwarm) {
  if (k <= 0 || m <= 0 || k + m > 256 || threads <= 0 || threads > 256 || nerased > m ||
      nobj <= 0 || max_passes <= 0 || structure < 0 || structure > 2)
    return ORC_E_PARAMS;
  uint64_t bs = orc_block_size(k, 8, size);
  bench_plan PE, PD;
  int rc = bench_plan_make(&PE, 0, k, m, NULL, 0);
  if (rc) return rc;
  rc = bench_plan_make(&PD, 1, k, m, erased, nerased);
  if (rc) { bench_plan_free(&PE); return rc; }
  const int simd = orc_simd_level();
  pthread_barrier_t start, done;
  pthread_barrier_init(&start, NULL, (unsigned)threads + 1);
  pthread_barrier_init(&done, NULL, (unsigned)threads + 1);
  volatile int stop = 0;
  bench_queue Q;
  Q.obj = calloc((size_t)nobj, sizeof(*Q.obj));
  Q.par = calloc((size_t)nobj, sizeof(*Q.par));
  Q.nobj = nobj;
  Q.next[0] = Q.next[1] = 0;
  pthread_barrier_init(&Q.mid, NULL, (unsigned)threads);
  pinned_worker *Ws = calloc((size_t)threads, sizeof(pinned_worker));
  pthread_t *th = calloc((size_t)threads, sizeof(pthread_t));
  for (int t = 0; t < threads; t++) {
    pinned_worker *W = &Ws[t];
    W->src = src; W->src_stride = src_stride; W->cpu = cpus ? cpus[t] : -1;
    W->start = &start; W->done = &done; W->stop = &stop; W->q = &Q;
    W->o0 = (int)((long long)nobj * t / threads);
    bench_job *E = &W->enc, *D = &W->dec;
    E->op = 0; E->k = k; E->m = m; E->nout = PE.nout; E->simd = simd; E->size = size; E->bs = bs;
    E->o0 = (int)((long long)nobj * t / threads);
    E->o1 = (int)((long long)nobj * (t + 1) / threads);
    E->tbl = PE.tbl; E->mats = PE.mats; E->want = PE.want; E->surv = PE.surv;
    E->coef = PE.coef; E->structure = structure;
    *D = *E;
    D->op = 1; D->nout = PD.nout; D->tbl = PD.tbl; D->mats = PD.mats; D->want = PD.want;
    D->surv = PD.surv; D->coef = PD.coef;
    pthread_create(&th[t], NULL, pinned_main, W);
  }
  /* round 0 (untimed): the first touch is done and the caches are warm.
   * The main thread resets the queue's counters between rounds, while every
   * worker waits at `start`. */
  int np = 0, any_err = 0;
  pthread_barrier_wait(&start);
  pthread_barrier_wait(&done);
  for (int t = 0; t < threads; t++) any_err |= Ws[t].err;
  double t_all = 0.0;
  /* one pass: whole rounds until pass_s has elapsed; its GiB/s */
#define ORC_PASS(dt_out, rate_out)                                                   \
  do {                                                                               \
    double t0_ = now_s(), dt_;                                                       \
    int reps_ = 0;                                                                   \
    do {                                                                             \
      Q.next[0] = Q.next[1] = 0;                                                     \
      pthread_barrier_wait(&start);                                                  \
      pthread_barrier_wait(&done);                                                   \
      reps_++;                                                                       \
      dt_ = now_s() - t0_;                                                           \
    } while (dt_ < pass_s);                                                          \
    (dt_out) = dt_;                                                                  \
    (rate_out) = 2.0 * (double)nobj * (double)size * reps_ / dt_ / (double)(1u << 30); \
  } while (0)
  /* untimed warm-up passes (the host ramps: a shared box's first passes of a
   * run read up to 25 % low, profiles/r04_s3_bench.log): until two
   * consecutive passes agree within 3 % or warm_s has elapsed */
  int nw = 0;
  for (double tw = 0.0; !any_err && warm_s > 0.0 && tw < warm_s;) {
    double dt, r;
    ORC_PASS(dt, r);
    tw += dt;
    if (warm_rates && nw < max_warm) warm_rates[nw] = r;
    nw++;
    if (nw >= 2 && warm_rates && nw <= max_warm &&
        fabs(r - warm_rates[nw - 2]) <= 0.03 * warm_rates[nw - 2])
      break;
  }
  if (nwarm) *nwarm = nw < max_warm ? nw : max_warm;
  while (!any_err && np < max_passes && (t_all < total_s || np < min_passes)) {
    const long long th0 = throttled_s ? cgroup_throttled_us() : -1;
    double dt, r;
    ORC_PASS(dt, r);
    t_all += dt;
    if (throttled_s) {
      const long long th1 = cgroup_throttled_us();
      throttled_s[np] = th0 < 0 || th1 < 0 ? -1.0 : (double)(th1 - th0) * 1e-6;
    }
    rates[np++] = r;
  }
#undef ORC_PASS
  stop = 1;
  pthread_barrier_wait(&start);
  int err = 0;
  for (int t = 0; t < threads; t++) {
    pthread_join(th[t], NULL);
    pinned_worker *W = &Ws[t];
    err |= W->err;
    const int n = W->enc.o1;
    if (parity_out && W->par)
      memcpy(parity_out + (uint64_t)((long long)nobj * t / threads) * m * bs, W->par,
             (uint64_t)n * m * bs);
    free(W->objs); free(W->par); free(W->tail);
  }
  free(Ws); free(th);
  free((void *)Q.obj); free(Q.par);
  pthread_barrier_destroy(&Q.mid);
  pthread_barrier_destroy(&start);
  pthread_barrier_destroy(&done);
  bench_plan_free(&PE);
  bench_plan_free(&PD);
  return err ? ORC_E_PARAMS : np;
}
