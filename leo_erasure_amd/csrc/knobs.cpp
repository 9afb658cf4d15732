// knobs.cpp — see knobs.hpp.
#include "knobs.hpp"

#ifdef LEOEC_MEASURE
#include <atomic>
#include <cstdlib>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <string_view>
#include <vector>
#endif

namespace leoec {

#ifndef LEOEC_MEASURE

const Knobs& knobs() {
  static const Knobs k;  // the shipped forms; the environment is never read
  return k;
}

#else

namespace {

// Overrides set through leoec_measure_set_knob (the form-parity tests):
// they take precedence over the environment, which is only read, never
// written, so no test mutates the process environment while library or HIP
// runtime threads run.  Guarded by g_mu.
std::map<std::string, std::string>& overrides() {
  static auto* m = new std::map<std::string, std::string>;
  return *m;
}

const char* lookup(const char* name) {
  const auto& o = overrides();
  const auto it = o.find(name);
  return it != o.end() ? it->second.c_str() : std::getenv(name);
}

int env_int(const char* name, int dflt) {
  const char* e = lookup(name);
  return e ? std::atoi(e) : dflt;
}

// Every snapshot ever published, kept (reachable) for the process: a
// launch may still read an older one.  Guarded by g_mu.
std::vector<std::unique_ptr<const Knobs>>& snapshots() {
  static auto* v = new std::vector<std::unique_ptr<const Knobs>>;
  return *v;
}

const Knobs* read_env() {
  Knobs* k = new Knobs;
  snapshots().emplace_back(k);
  k->bitmatrix = env_int("LEOEC_BITMATRIX", k->bitmatrix);
  if (const char* e = lookup("LEOEC_HOST_STAGING")) {
    const std::string_view v(e);
    k->host_staging = v == "pageable" ? 1 : v == "gather" ? 2 : v == "pinned" ? 3
                      : v == "zerocopy" ? 4 : 0;
  }
  k->stage_chunk_kib = env_int("LEOEC_STAGE_CHUNK_KIB", k->stage_chunk_kib);
  k->zc_chunks = env_int("LEOEC_ZC_CHUNKS", k->zc_chunks);
  k->host_batch = env_int("LEOEC_HOST_BATCH", k->host_batch);
  k->batch_window_us = env_int("LEOEC_BATCH_WINDOW_US", k->batch_window_us);
  k->hostq_depth = env_int("LEOEC_HOSTQ_DEPTH", k->hostq_depth);
  if (k->hostq_depth < 1 || k->hostq_depth > 4) k->hostq_depth = 3;  // 5 slots: one stays open
  k->hostq_sync = env_int("LEOEC_HOSTQ_SYNC", k->hostq_sync);
  k->hostq_streams = env_int("LEOEC_HOSTQ_STREAMS", k->hostq_streams);
  k->hostq_split_kib = env_int("LEOEC_HOSTQ_SPLIT_KIB", k->hostq_split_kib);
  k->hostq_slot_kib = env_int("LEOEC_HOSTQ_SLOT_KIB", k->hostq_slot_kib);
  k->hostq_eager = env_int("LEOEC_HOSTQ_EAGER", k->hostq_eager);
  k->hostq_close = env_int("LEOEC_HOSTQ_CLOSE", k->hostq_close);
  k->hostq_direct = env_int("LEOEC_HOSTQ_DIRECT", k->hostq_direct);
  k->hostq_direct_map = env_int("LEOEC_HOSTQ_DIRECT_MAP", k->hostq_direct_map);
  k->hostq_lanes = env_int("LEOEC_HOSTQ_LANES", k->hostq_lanes);
  k->hostq_zc = env_int("LEOEC_HOSTQ_ZC", k->hostq_zc);
  k->hostq_ntcopy = env_int("LEOEC_HOSTQ_NTCOPY", k->hostq_ntcopy);
  k->hostq_survivors = env_int("LEOEC_HOSTQ_SURVIVORS", k->hostq_survivors);
  k->hostq_wake = env_int("LEOEC_HOSTQ_WAKE", k->hostq_wake);
  k->hostq_fail_bs = env_int("LEOEC_HOSTQ_FAIL_BS", k->hostq_fail_bs);
  k->gf8_variant = env_int("LEOEC_GF8_VARIANT", k->gf8_variant);
  k->gf8_tmap = env_int("LEOEC_GF8_TMAP", k->gf8_tmap);
  k->gf8_tmap_set = lookup("LEOEC_GF8_TMAP") != nullptr;
  k->gf8_wg = env_int("LEOEC_GF8_WG", k->gf8_wg);
  k->gf8_tgroup = env_int("LEOEC_GF8_TGROUP", k->gf8_tgroup);
  k->gfw_form = env_int("LEOEC_GFW_FORM", k->gfw_form);
  k->gfp_cpt = env_int("LEOEC_GFP_CPT", k->gfp_cpt);
  k->gfp_bpc = env_int("LEOEC_GFP_BPC", k->gfp_bpc);
  k->bit_form = env_int("LEOEC_BIT_FORM", k->bit_form);
  if (k->bit_form < 0 || k->bit_form > 9) k->bit_form = 4;
  k->lib_form = env_int("LEOEC_LIB_FORM", k->lib_form);
  k->lib_la = env_int("LEOEC_LIB_LA", k->lib_la);
  k->lib_wg = env_int("LEOEC_LIB_WG", k->lib_wg);
  k->lib_dec_wg = env_int("LEOEC_LIB_DEC_WG", k->lib_dec_wg);
  k->lib_xmap = env_int("LEOEC_LIB_XMAP", k->lib_xmap);
  k->lib_buf = env_int("LEOEC_LIB_BUF", k->lib_buf);
  k->lib_dec_la = env_int("LEOEC_LIB_DEC_LA", k->lib_dec_la);
  k->lib_dec_cod = env_int("LEOEC_LIB_DEC_COD", k->lib_dec_cod);
  k->gfbit_xmap = env_int("LEOEC_GFBIT_XMAP", k->gfbit_xmap);
  k->gfbit_lw = env_int("LEOEC_GFBIT_LW", k->gfbit_lw);
  k->gfbit_pf = env_int("LEOEC_GFBIT_PF", k->gfbit_pf);
  k->gfbit_wg = env_int("LEOEC_GFBIT_WG", k->gfbit_wg);
  k->gfbit_ceil = env_int("LEOEC_GFBIT_CEIL", k->gfbit_ceil);
  k->gfbit_lds = env_int("LEOEC_GFBIT_LDS", k->gfbit_lds);
  k->gfbit_form = env_int("LEOEC_GFBIT_FORM", k->gfbit_form);
  k->gfbk_min_mib = env_int("LEOEC_GFBK_MIN_MIB", k->gfbk_min_mib);
  k->gfbit_waves = env_int("LEOEC_GFBIT_WAVES", k->gfbit_waves);
  k->gfbit_cbm = env_int("LEOEC_GFBIT_CBM", k->gfbit_cbm);
  k->gfs_mode = env_int("LEOEC_GFS_MODE", k->gfs_mode);
  k->gfs_pf = env_int("LEOEC_GFS_PF", k->gfs_pf);
  return k;
}

std::atomic<const Knobs*> g_knobs{nullptr};
std::mutex g_mu;

}  // namespace

const Knobs& knobs() {
  const Knobs* k = g_knobs.load(std::memory_order_acquire);
  if (k) return *k;
  std::lock_guard<std::mutex> lock(g_mu);
  k = g_knobs.load(std::memory_order_relaxed);
  if (!k) {
    k = read_env();
    g_knobs.store(k, std::memory_order_release);
  }
  return *k;
}

}  // namespace leoec

// Measurement build only: re-read the LEOEC_* variables and overrides.
// Earlier snapshots stay valid (they are never freed), so a concurrent launch
// sees either the old or the new set.
extern "C" __attribute__((visibility("default"))) void leoec_measure_reload(void) {
  std::lock_guard<std::mutex> lock(leoec::g_mu);
  leoec::g_knobs.store(leoec::read_env(), std::memory_order_release);
}

// Measurement build only: set knob `name` (an LEOEC_* name) to `value`, or
// drop its override with value == NULL (the environment's value, if any,
// applies again), and publish a new snapshot.  Returns 0, or -1 for a name
// that is not an LEOEC_* knob.
extern "C" __attribute__((visibility("default"))) int leoec_measure_set_knob(const char* name,
                                                                            const char* value) {
  if (!name || std::string_view(name).rfind("LEOEC_", 0) != 0) return -1;
  std::lock_guard<std::mutex> lock(leoec::g_mu);
  if (value)
    leoec::overrides()[name] = value;
  else
    leoec::overrides().erase(name);
  leoec::g_knobs.store(leoec::read_env(), std::memory_order_release);
  return 0;
}

// Measurement build only: drop every override set by leoec_measure_set_knob.
extern "C" __attribute__((visibility("default"))) void leoec_measure_reset_knobs(void) {
  std::lock_guard<std::mutex> lock(leoec::g_mu);
  leoec::overrides().clear();
  leoec::g_knobs.store(leoec::read_env(), std::memory_order_release);
}

namespace leoec {
#endif

}  // namespace leoec
