/*
 * leoec.h — C ABI of the MI355X-native leo_erasure engine (libleoec.so).
 *
 * This is the drop-in seam for the reference's NIF (c_src/leo_erasure_nif.cpp).
 * The reference NIF exports gf_init/0, encode/4, decode/5, repair/5
 * (c_src/leo_erasure_nif.cpp:346-353) and implements them with C++ coder
 * classes over Jerasure / ISA-L (c_src/{rs,cauchy,liberation,irs}coding.cpp).
 * Each host entry point below is what that NIF binds once its arithmetic is
 * moved onto the GPU; the NIF keeps parsing terms and building binaries
 * (see INTEGRATION.md for the shim).  The *_dev entry points are the
 * device-resident, batched form of the same operations.
 *
 * Conventions
 *   - plain pointers and sizes only; no exceptions cross this boundary;
 *   - every function returns LEOEC_OK (0) or a negative leoec_status;
 *     leoec_strerror() gives the reference's message text for it;
 *   - reentrant and thread-safe: concurrent callers (the basho_bench t4
 *     configuration) each get their own HIP stream and staging buffers;
 *   - the GF arithmetic always runs on the GPU (HIP, gfx950); a missing or
 *     unusable device is reported as LEOEC_E_NO_DEVICE, never computed on CPU.
 */
#ifndef LEOEC_H
#define LEOEC_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* The library is built with hidden visibility; everything declared here is
 * its export table. */
#pragma GCC visibility push(default)

/* Coding classes — same numbering as CodingType (c_src/leo_erasure_nif.cpp:36-42);
 * atom names vandrs | cauchyrs | liberation | isars (nif.cpp:61-72). */
enum leoec_coding {
  LEOEC_CAUCHYRS = 1,
  LEOEC_VANDRS = 2,
  LEOEC_LIBERATION = 3,
  LEOEC_ISARS = 4,
};

enum leoec_status {
  LEOEC_OK = 0,
  LEOEC_E_INVALID_CODING = -1,      /* "Invalid Coding"                           nif.cpp:55,71   */
  LEOEC_E_PARAMS = -2,              /* "Invalid Coding Parameters"                rscoding.cpp:31 */
  LEOEC_E_PARAMS_W_RS = -3,         /* "Invalid Coding Parameters (w = 8/16/32)"  rscoding.cpp:33 */
  LEOEC_E_PARAMS_LARGER_W = -4,     /* "Invalid Coding Parameters (larger w)"     cauchycoding.cpp:34 */
  LEOEC_E_PARAMS_M2 = -5,           /* "Invalid Coding Parameters (m = 2)"        liberationcoding.cpp:31 */
  LEOEC_E_PARAMS_K_LE_W = -6,       /* "Invalid Coding Parameters (k <= w)"       liberationcoding.cpp:33 */
  LEOEC_E_PARAMS_W_PRIME = -7,      /* "Invalid Coding Parameters (w is prime)"   liberationcoding.cpp:35 */
  LEOEC_E_PARAMS_W8 = -8,           /* "Invalid Coding Parameters (w = 8)"        irscoding.cpp:36 */
  LEOEC_E_NOT_ENOUGH_BLOCKS = -9,   /* "Not Enough Blocks"                        rscoding.cpp:91 */
  LEOEC_E_NOT_UNIQUE = -10,         /* "Blocks should be unique"                  rscoding.cpp:93 */
  LEOEC_E_NON_INVERTIBLE = -11,     /* "Non Invertible"                           irscoding.cpp:203 */
  LEOEC_E_BAD_ID = -12,             /* block / repair id outside 0..k+m-1 (reference: UB) */
  LEOEC_E_BAD_SIZE = -13,           /* inconsistent block size or object size > k*bs (reference: UB) */
  LEOEC_E_UNSUPPORTED = -14,        /* parameters the field / matrix construction cannot serve */
  LEOEC_E_NOMEM = -15,              /* host or device allocation failed (reference: terminate) */
  LEOEC_E_NO_DEVICE = -16,          /* no usable gfx950 HIP device */
  LEOEC_E_HIP = -17,                /* a HIP runtime call failed */
  LEOEC_E_ARG = -18,                /* NULL pointer / negative count / misaligned device buffer */
};

/* Message text for a status (static storage). */
const char *leoec_strerror(int status);

/* ---- the NIF surface ---------------------------------------------------- */

/* gf_init/0 (c_src/leo_erasure_nif.cpp:122-128): build the GF(2^8/16/32)
 * host tables, open the HIP device and warm the caller's current device once
 * (its hardware queues, the runtime's pageable-copy staging, every kernel
 * code object, the device's batching queue, pools of streams and mapped
 * buffers for other threads' first calls: 0.2-0.4 s) so the VM's first calls
 * are not charged for them.  Idempotent; other calls open the device lazily
 * (without the warm-up). */
int leoec_gf_init(void);

/* Coder::checkParams of the class (rscoding.cpp:29-34, cauchycoding.cpp:30-35,
 * liberationcoding.cpp:29-36, irscoding.cpp:32-37; factory nif.cpp:44-72). */
int leoec_check_params(int coding, int k, int m, int w);

/* Stripe geometry (c_src/common.cpp:24-33 + rscoding.cpp:44-54):
 *   block_size = roundTo(roundTo(size, k*w) / (k*w), 16) * w
 *   filled     = number of whole blocks that alias the input (<= k)      */
int leoec_layout(int coding, int k, int m, int w, uint64_t size, uint64_t *block_size,
                 int *filled);

/* encode/4 (nif.cpp:130-166 -> RSCoding::doEncode rscoding.cpp:36-85 and the
 * other classes' doEncode).  Writes blocks filled..k+m-1 — the zero-padded tail
 * data block(s) followed by the m coding blocks — contiguously into `out`
 * ((k+m-filled)*block_size bytes), exactly the bytes of the reference's
 * freshly allocated binary; blocks 0..filled-1 are the input itself
 * (zero-copy sub-binaries in the NIF). */
int leoec_encode(int coding, int k, int m, int w, const uint8_t *obj, uint64_t size,
                 uint8_t *out, uint64_t out_size);

/* decode/5 (nif.cpp:169-249 -> doDecode, e.g. rscoding.cpp:87-154).
 * blocks[i] (block_size bytes) has id ids[i]; any order, >= k unique ids.
 * Writes the first `size` bytes of D0..Dk-1 to `out`. */
int leoec_decode(int coding, int k, int m, int w, const uint8_t *const *blocks, const int *ids,
                 int nblocks, uint64_t block_size, uint64_t size, uint8_t *out);

/* repair/5 (nif.cpp:252-344 -> doRepair, e.g. rscoding.cpp:156-211).
 * Writes the blocks repair_ids[0..nrepair-1], in that order, to
 * out + r*block_size. */
int leoec_repair(int coding, int k, int m, int w, const uint8_t *const *blocks, const int *ids,
                 int nblocks, uint64_t block_size, const int *repair_ids, int nrepair,
                 uint8_t *out);

/* ---- device-resident, batched ------------------------------------------- *
 * All pointers are HIP device pointers, 16-byte aligned, strides multiples
 * of 16; work is enqueued on `stream` (a hipStream_t, NULL = default stream)
 * and the call returns without synchronising.  `nobj` objects are processed
 * per call; object o's block j lives at base + o*stride + j*block_size.
 * Strides cover a whole row (obj_stride >= size, parity_stride >=
 * m*block_size, block/out strides >= block_size) for every nobj >= 1;
 * otherwise LEOEC_E_ARG.  The buffers themselves cannot be checked here:
 * they must hold nobj rows.                                                */

/* Encode nobj objects of `size` bytes each, stored at objs + o*obj_stride
 * (the unpadded object; bytes past `size` inside the last data block are
 * read as zero and never touched).  Coding block i of object o is written to
 * parity + o*parity_stride + i*block_size. */
int leoec_encode_dev(int coding, int k, int m, int w, const uint8_t *objs, uint64_t obj_stride,
                     uint64_t size, uint64_t nobj, uint8_t *parity, uint64_t parity_stride,
                     void *stream);

/* In-place decode: the surviving data blocks are in objs (as for encode),
 * the coding blocks in parity; the data blocks listed in erased[] are rebuilt
 * into objs (clipped to `size`).  Erased coding ids are allowed and mean
 * "not a survivor".  Survivor choice follows the reference (first k intact
 * ids ascending; isars: data survivors ascending, then coding). */
int leoec_decode_dev(int coding, int k, int m, int w, uint8_t *objs, uint64_t obj_stride,
                     uint64_t size, uint64_t nobj, const uint8_t *parity, uint64_t parity_stride,
                     const int *erased, int nerased, void *stream);

/* Generic repair: block id b of object o is at blocks[b] + o*block_stride
 * (blocks[b] == NULL: missing), each block_size bytes.  Rebuilds repair_ids
 * into out[r] + o*out_stride. */
int leoec_repair_dev(int coding, int k, int m, int w, const uint8_t *const *blocks,
                     uint64_t block_stride, uint64_t block_size, uint64_t nobj,
                     const int *repair_ids, int nrepair, uint8_t *const *out,
                     uint64_t out_stride, void *stream);

/* ---- introspection ------------------------------------------------------ */

/* Coding matrix the engine uses: m*k words (GF classes) or a (m*w) x (k*w)
 * 0/1 bitmatrix as bytes (cauchyrs, liberation).  *n_out = entries written. */
int leoec_coding_matrix(int coding, int k, int m, int w, uint32_t *out, int cap, int *n_out);

/* Device ordinal the calling thread's device-resident calls (*_dev) use,
 * or a negative status. */
int leoec_device(void);

/* Host-memory calls (leoec_encode / _decode / _repair) run on the calling
 * thread's current HIP device by default (each device has its own batching
 * queue, its dispatcher lane).  Returns the number of lanes (one per gfx950
 * device visible to the process) and writes the device ordinal of lane i to
 * devices[i] for i < cap (devices may be NULL), or a negative status.
 * (No reference counterpart: the reference is CPU-only.) */
int leoec_host_lanes(int *devices, int cap);

/* Opt in to spreading host-memory calls over several devices: with n > 0,
 * each later call goes to the device of devices[0..n-1] whose lane has the
 * fewest calls in progress (its own queue and PCIe link), and the caller's
 * current device is left as it was; n == 0 restores the default (the
 * caller's current device).  Every ordinal must be a gfx950 device visible
 * to the process (else LEOEC_E_NO_DEVICE, and the setting is unchanged).
 * Returns the number of devices in the set.  Only the devices of the set get
 * queues and pinned arenas (5 x 32 MiB pinned + 5 x 32 MiB device each), and
 * each of them is warmed before this returns, as gf_init warms the caller's
 * device (its hardware queues, code objects, batching queue and pools, one
 * thread per device: ~0.3 s once), so no device's first call pays that.
 * (No reference counterpart: the reference is CPU-only.) */
int leoec_host_spread(const int *devices, int n);

/* Library version string. */
const char *leoec_version(void);

#pragma GCC visibility pop

#ifdef __cplusplus
}
#endif
#endif /* LEOEC_H */
