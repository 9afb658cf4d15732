/*
 * leoec_oracle.h — CPU restatement of leo_erasure's coding arithmetic.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing under oracle/ is linked into, loaded by,
 * or called from the product (leo_erasure_amd/).  Only tests/, the smoke()
 * entry of __graft_entry__.py and the cpu_baseline leg of bench.py may use it,
 * and only as the checker / the reported CPU baseline.
 *
 * What it restates (the reference links these libraries but does not vendor
 * them; they are git-cloned at build time, unpinned — c_src/build_deps.sh:48-60):
 *   - gf-complete default fields (w = 1..32, default primitive polynomials),
 *   - Jerasure 2.0 reed_sol_vandermonde_coding_matrix, cauchy_original /
 *     improve / good_general (incl. the m = 2 "cbest" rows), liberation
 *     bitmatrix, matrix->bitmatrix expansion, jerasure_matrix_encode /
 *     decode / decode_selected and the bitmatrix (schedule) encode / decode,
 *   - ISA-L gf_gen_cauchy1_matrix, gf_invert_matrix, ec_encode_data,
 *   - leo_erasure's stripe geometry and NIF-level semantics
 *     (c_src/common.cpp:24-33, c_src/rscoding.cpp:36-211,
 *      c_src/cauchycoding.cpp:29-213, c_src/liberationcoding.cpp:29-208,
 *      c_src/irscoding.cpp:32-220).
 * Pins: see tests/test_oracle.py (KATs) and DESIGN.md §Oracle.
 *
 * PARITY UNPINNED (strict sense): the reference's tests hold no known-answer
 * vectors and the reference cannot be built or run here (no Erlang/OTP, its
 * Jerasure / gf-complete / ISA-L dependencies are absent), so no vector in
 * tests/ comes from the reference itself.  The restatement is pinned by
 * recalled public KATs (Jerasure manual reed_sol_01 7 7 8, cbest_2..5), an
 * independent numpy restatement, and the reference's round-trip properties.
 */
#ifndef LEOEC_ORACLE_H
#define LEOEC_ORACLE_H
#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

/* coding classes: same numbering as CodingType (c_src/leo_erasure_nif.cpp:36-42) */
enum { ORC_CAUCHYRS = 1, ORC_VANDRS = 2, ORC_LIBERATION = 3, ORC_ISARS = 4 };

/* status codes: same numbering as include/leoec.h (checked by tests) */
enum {
  ORC_OK = 0,
  ORC_E_INVALID_CODING = -1,
  ORC_E_PARAMS = -2,            /* "Invalid Coding Parameters" */
  ORC_E_PARAMS_W_RS = -3,       /* "Invalid Coding Parameters (w = 8/16/32)" */
  ORC_E_PARAMS_LARGER_W = -4,   /* "Invalid Coding Parameters (larger w)" */
  ORC_E_PARAMS_M2 = -5,         /* "Invalid Coding Parameters (m = 2)" */
  ORC_E_PARAMS_K_LE_W = -6,     /* "Invalid Coding Parameters (k <= w)" */
  ORC_E_PARAMS_W_PRIME = -7,    /* "Invalid Coding Parameters (w is prime)" */
  ORC_E_PARAMS_W8 = -8,         /* "Invalid Coding Parameters (w = 8)" */
  ORC_E_NOT_ENOUGH = -9,        /* "Not Enough Blocks" */
  ORC_E_NOT_UNIQUE = -10,       /* "Blocks should be unique" */
  ORC_E_NON_INVERTIBLE = -11,   /* "Non Invertible" */
  ORC_E_BAD_ID = -12,
  ORC_E_BAD_SIZE = -13,
  ORC_E_UNSUPPORTED = -14,
  ORC_E_NOMEM = -15,
};

/* ---- field ---- */
uint64_t orc_prim_poly(int w);                 /* incl. the x^w term; 0 for w = 32 form see .c */
uint32_t orc_gf_mul(uint32_t a, uint32_t b, int w);
uint32_t orc_gf_inv(uint32_t a, int w);
uint32_t orc_gf_div(uint32_t a, uint32_t b, int w);

/* ---- matrices ---- */
int orc_vandermonde_coding_matrix(int k, int m, int w, uint32_t *out);      /* m*k */
int orc_cauchy_original_coding_matrix(int k, int m, int w, uint32_t *out);  /* m*k */
void orc_cauchy_improve_coding_matrix(int k, int m, int w, uint32_t *mat);
int orc_cauchy_good_general_coding_matrix(int k, int m, int w, uint32_t *out);
int orc_cauchy_n_ones(uint32_t n, int w);
int orc_cbest_row(int w, int k, uint32_t *out);       /* first k cbest entries */
int orc_liberation_coding_bitmatrix(int k, int w, uint8_t *out);            /* 2w x kw */
int orc_matrix_to_bitmatrix(int k, int m, int w, const uint32_t *mat, uint8_t *out); /* mw x kw */
int orc_isal_gen_cauchy1_matrix(int rows, int k, uint8_t *out);             /* rows*k */
int orc_isal_invert_matrix(const uint8_t *in, uint8_t *out, int n);

/* ---- geometry ---- */
uint64_t orc_round_to(uint64_t n, uint64_t multiple);
uint64_t orc_block_size(int k, int w, uint64_t size);
int orc_check_params(int coding, int k, int m, int w);

/* ---- NIF-level semantics ----
 * encode: blocks = (k+m)*bs bytes, block i at blocks + i*bs.
 * decode: blocks[i] has id ids[i], all of size bs; out gets `size` bytes.
 * repair: out gets nrep*bs bytes in rep order. */
int orc_encode(int coding, int k, int m, int w, const uint8_t *obj, uint64_t size,
               uint8_t *blocks);
int orc_decode(int coding, int k, int m, int w, const uint8_t *const *blocks,
               const int *ids, int n, uint64_t bs, uint64_t size, uint8_t *out);
int orc_repair(int coding, int k, int m, int w, const uint8_t *const *blocks,
               const int *ids, int n, uint64_t bs, const int *rep, int nrep,
               uint8_t *out);

/* ---- CPU baseline (ISA-L technique: split 4-bit tables, PSHUFB) ----
 * Encodes (op 0) or decodes-with-erasures (op 1, erased data ids given) `nobj`
 * objects of `size` bytes laid out at `obj_stride`, vandrs(k,m,8), using
 * `threads` pthreads.  Parity goes to parity + o*m*bs.  Returns 0 or <0. */
int orc_bench_rs8(int op, int k, int m, const uint8_t *objs, uint64_t obj_stride,
                  uint64_t size, int nobj, uint8_t *parity, const int *erased,
                  int nerased, int threads, int force_scalar);
/* bench.py's timed baseline: pinned workers, per-worker first-touched
 * sample slices, passes of >= pass_s s; returns the pass count (rates[]). */
int orc_bench_rs8_pinned(int k, int m, const uint8_t *src, uint64_t src_stride, uint64_t size,
                         int nobj, const int *erased, int nerased, int threads, const int *cpus,
                         double pass_s, double total_s, int min_passes, double *rates,
                         int max_passes, uint8_t *parity_out, int structure,
                         double *throttled_s, double warm_s, double *warm_rates, int max_warm,
                         int *nwarm);
int orc_simd_level(void);   /* 0 scalar, 2 avx2 (PSHUFB), 3 avx512bw+gfni (affine) */

#ifdef __cplusplus
}
#endif
#endif
