// knobs.hpp — kernel-form and staging-form selectors.
//
// The product library (libleoec.so) ships one form of every kernel and one
// host-staging policy: knobs() returns these compiled-in defaults and the
// library never reads the environment.  The measurement build
// (libleoec_measure.so, `make measure`, -DLEOEC_MEASURE) also compiles the
// alternative forms kept for A/B runs and parity checks, and fills the knobs
// from LEOEC_* environment variables once, at first use (thread-safe);
// leoec_measure_reload() re-reads them for a test that changes a variable.
#pragma once

namespace leoec {

struct Knobs {
  // engine.cpp
  int bitmatrix = 0;         // LEOEC_BITMATRIX=1: cauchyrs through the generic bitmatrix kernel
  int host_staging = 0;      // LEOEC_HOST_STAGING: 0 auto, 1 pageable, 2 gather, 3 pinned ring,
                             //   4 zero-copy (kernels on pinned, device-mapped host memory)
  int stage_chunk_kib = 256; // LEOEC_STAGE_CHUNK_KIB: pinned-ring chunk
  int zc_chunks = 2;         // LEOEC_ZC_CHUNKS: a per-thread zero-copy call of a GF(2^w) map
                             //   in this many column chunks, packing chunk c + 1 while
                             //   chunk c's launch runs and unpacking each as it completes
                             //   (shipped at 2 since round 4: a lone 1 MiB encode 79.6 ->
                             //   70.2 us, profiles/r04_s14_lone_*.log; 3 and 4 lose)
  int host_batch = 1;        // LEOEC_HOST_BATCH=0: host calls take the per-thread path only
  int batch_window_us = 0;   // LEOEC_BATCH_WINDOW_US: hold an idle-GPU batch open this long
  int hostq_depth = 3;       // LEOEC_HOSTQ_DEPTH: batches on the GPU at once
  int hostq_streams = 1;     // LEOEC_HOSTQ_STREAMS: 1 a batch's H2D / D2H on the queue's two copy
                             // streams (shipped), 0 everything on the slot's stream
  int hostq_split_kib = 1024;  // LEOEC_HOSTQ_SPLIT_KIB: batches with less input than this stay on
                             // the slot's stream (their cross-stream events cost more than the
                             // link's overlap gives: 16 / 64 KiB objects -5 % split,
                             // profiles/r05_s39_small_streams*.log)
  int hostq_slot_kib = 16384;  // LEOEC_HOSTQ_SLOT_KIB: input (and output) bytes a batch may hold
                             //   (at most the 16 MiB arenas; a lone job larger than this still
                             //   takes an empty slot)
  int hostq_eager = 0;       // LEOEC_HOSTQ_EAGER=1: the caller whose reservation leaves no room for
                             //   another job of its size hands the slot to the worker at once
                             //   (0: the next caller finds it full, or the worker closes it when
                             //   the previous batch's H2D ends, Knobs::hostq_close)
  int hostq_sync = 1;        // LEOEC_HOSTQ_SYNC: 1 poll events (hipEventQuery + yield),
                             //   0 hipEventSynchronize, 2 the same on blocking-sync events
  int hostq_close = 1;       // LEOEC_HOSTQ_CLOSE: 1 close a batch when the previous H2D is
                             //   done, 0 as soon as the GPU has room
  int hostq_direct = 16;     // LEOEC_HOSTQ_DIRECT: encode calls that may take the per-thread
                             //   path while the queue is idle (0: every call batched)
  int hostq_direct_map = 8;  // LEOEC_HOSTQ_DIRECT_MAP: the same for decode / repair (their
                             //   per-thread path gathers k buffers: it tops out sooner)
                             //   (round 5: 16 / 8, was 4 / 2: encode +21 % at 8 callers,
                             //   +17 % at 16, decode +30 % at 4, +27 % at 8, 32 callers
                             //   unchanged; profiles/r05_s26_*.log, three rotated rounds)
  int hostq_fail_bs = 0;     // LEOEC_HOSTQ_FAIL_BS: batched launches of this block size report
                             //   a HIP error (fault injection: per-job status)
  int hostq_zc = 0;          // LEOEC_HOSTQ_ZC=1: batches without DMA copies (kernels on the
                             //   pinned, device-mapped arenas)
  int hostq_lanes = 0;       // LEOEC_HOSTQ_LANES: dispatcher lanes (0: one per gfx950 device;
                             //   N: N lanes, lane i on device i % devices)
  int hostq_ntcopy = 1;      // LEOEC_HOSTQ_NTCOPY=0: callers pack gathered inputs (decode /
                             //   repair) into the pinned buffers with memcpy instead of
                             //   non-temporal stores (host_copy.hpp; shipped since round 4)
  int hostq_wake = 1;        // LEOEC_HOSTQ_WAKE: 1 targeted wake-ups (a batch's callers on
                             //   its slot's condition variable; the worker woken by a
                             //   slot's first reservation only; slot-free waiters counted),
                             //   0 the round-4 broadcasts (every waiting caller per batch)
  int hostq_survivors = 1;   // LEOEC_HOSTQ_SURVIVORS: where a batched decode copies its
                             //   surviving data blocks into the output: 1 while its batch
                             //   is on the GPU, 0 before joining the batch, 2 after its
                             //   outputs are unpacked (the slot is freed sooner)
  // kernels.hip / kernels_impl.hpp
  int gf8_variant = 0;       // LEOEC_GF8_VARIANT: gf8_apply<10,4> variant (gf8_exp.hip)
  int gf8_tmap = 0;          // LEOEC_GF8_TMAP: gf8_apply workgroup -> tile order
  bool gf8_tmap_set = false; //   (given: no automatic xcd_obj_map)
  int gf8_wg = 0;            // LEOEC_GF8_WG=64|256: force the gf8 tile width
  int gf8_tgroup = 0;        // LEOEC_GF8_TGROUP: tiles per XCD group of tile map 4
  int gfw_form = 3;          // LEOEC_GFW_FORM: w=16/32 kernel (3 bitsliced gfs_apply,
                             //   0 byte-plane gfp_apply, 1/2 older forms)
  int gfp_cpt = 2;           // LEOEC_GFP_CPT: gfp_apply 16-byte columns per lane
  int gfp_bpc = 64;          // LEOEC_GFP_BPC: gfp_apply resident blocks per CU
  int bit_form = 4;          // LEOEC_BIT_FORM: bitmatrix kernel form
  int lib_form = 1;          // LEOEC_LIB_FORM=0: liberation through the generic bitmatrix kernel
  int lib_la = 2;            // LEOEC_LIB_LA: lib_apply packet look-ahead
  int lib_wg = 64;           // LEOEC_LIB_WG=256: lib_apply with 256-lane workgroups (4 KiB tiles)
  int lib_dec_wg = 0;        // LEOEC_LIB_DEC_WG=64|256: the syndrome kernel's lanes (0: the
                             //   form's shipped width, 64 libb_dec_apply / 256 lib_dec_apply)
  int lib_xmap = 2;          // LEOEC_LIB_XMAP=0: liberation kernels without xcd_obj_map
  int lib_buf = -1;          // LEOEC_LIB_BUF: the liberation kernels with branch-free raw buffer
                             //   loads (libb_apply / libb_dec_apply, kernels_impl.hpp): -1 the
                             //   shipped policy (encode w >= 11, every syndrome decode), 1 always,
                             //   0 never (lib_apply / lib_dec_apply)
  int lib_dec_la = -1;       // LEOEC_LIB_DEC_LA: libb_dec_apply packet look-ahead (0: the block
                             //   form; -1: shipped, libb_dec_la(w, k))
  int lib_dec_cod = 1;       // LEOEC_LIB_DEC_COD=0: wanted coding blocks (repair of {data, P},
                             //   {Q}, ...) through the generic bitmatrix kernel, not syndromes
  // gfbit_inst.hip
  int gfbit_xmap = -1;       // LEOEC_GFBIT_XMAP: 0 off, 1 object-contiguous, unset auto
  int gfbit_lw = 2;          // LEOEC_GFBIT_LW: lane width (dwords per packet), w = 8
  int gfbit_pf = 1;          // LEOEC_GFBIT_PF: blocks of load look-ahead, w = 8 (gfbit_apply 0..3; gfb2 0 or 1)
  int gfbit_wg = 0;          // LEOEC_GFBIT_WG=64: 64-lane workgroups; 128: 16-byte lanes
  int gfbit_ceil = 0;        // LEOEC_GFBIT_CEIL: traffic-ceiling kernel (not a code)
  int gfbit_lds = 0;         // LEOEC_GFBIT_LDS=1: LDS-staged inputs
  int gfbit_waves = 0;       // LEOEC_GFBIT_WAVES=4|5: register cap (waves per SIMD), w = 8
  int gfs_pf = 1;            // LEOEC_GFS_PF=2: two inputs in flight (w = 16/32, 4 rows)
  int gfs_mode = 0;          // LEOEC_GFS_MODE=1|2: w = 32 timing forms (not a code)
  int gfbit_cbm = 0;         // LEOEC_GFBIT_CBM: cauchyrs(10,4,8) encode with its bitmatrix compiled
                             //   in (cbm_inst.hip): 0 off, 1 64 lanes 2 waves 16 packets in flight, 2 the same
                             //   with 10, 3 128 lanes, 4 64 lanes 3 waves 4 in flight, 5 256 lanes
  int gfbk_min_mib = -1;     // LEOEC_GFBK_MIN_MIB: launches of at least this many MiB of algorithmic
                             //   bytes take gfbk_apply (w = 8, K = 10, 4 rows; -1: the shipped
                             //   kGfbkMinBytes, gfbit_impl.hpp; a huge value: never)
  int gfbit_form = 0;        // LEOEC_GFBIT_FORM: 0 gfbit_apply (shipped), 1 gfb2_apply (buffer loads)
};

const Knobs& knobs();

#ifdef LEOEC_MEASURE
constexpr bool kMeasureBuild = true;
#else
constexpr bool kMeasureBuild = false;
#endif

}  // namespace leoec
