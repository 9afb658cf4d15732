// leo_erasure_nif.cpp — NIF shim binding the reference's Erlang module
// `leo_erasure` (src/leo_erasure.erl:171,194,245,249) to libleoec.so.
//
// Drop-in for c_src/leo_erasure_nif.cpp: same module name, the same four
// NIFs (gf_init/0, encode/4, decode/5, repair/5 — nif.cpp:346-353), the same
// argument checks in the same order and the same {error, Latin-1 string}
// returns.  The coder classes and Jerasure / ISA-L are replaced by leoec_*
// calls; the arithmetic runs on the GPU.  Differences from the reference are
// deliberate fixes: coder errors keep their text,
// {K,M,W} arity is checked, and the NIFs run on dirty schedulers so a GPU
// round trip never blocks a normal scheduler thread.
//
// load/3 (the reference has none, nif.cpp:353): the library alone runs a
// host-memory call on the calling scheduler thread's current HIP device,
// which for every scheduler of a VM is device 0.  So the shim spreads the
// VM's calls over every gfx950 device it can see by default (round 5; one
// VM per GPU, started with HIP_VISIBLE_DEVICES, sees just its own), and
// LEOEC_HOST_DEVICES overrides that before the VM starts: "all" (the
// default), a comma list of device ordinals, or "current" / "" for no
// spreading (each call on its scheduler thread's current device, the
// library's own rule).  load passes the set to leoec_host_spread (which
// warms every device of the set before returning), and calls then go to
// the least-loaded device of the set.  A malformed
// value fails the load, and so does a well-formed set naming a device the
// process cannot use (say "0,1,7" on a 2-GPU node: leoec_host_spread refuses
// it and would leave every call on the scheduler thread's current device);
// the message goes to stderr.  Without any gfx950 device the value is left
// to the data calls, which report LEOEC_E_NO_DEVICE as usual.
//
// -DLEOEC_NIF_REF_ERRORS reproduces the reference's error terms exactly: its
// coder exceptions are rethrown by value as std::exception
// (nif.cpp:80-83,94-97,108-111), so every coder / engine failure reads
// "std::exception", and a failed gf_init reads "Galois Initialization
// Failed! w=8" (nif.cpp:124).  The default keeps the engine's message.
//
// Built only where erl_nif.h exists:
//   c++ -O2 -fPIC -shared -DHAVE_ERL_NIF -I$ERL_ROOT/usr/include -I<repo>/include
//       leo_erasure_nif.cpp -L<repo>/leo_erasure_amd -lleoec -o priv/leo_erasure.so
// tests/nif_harness/ compiles this file against a test-double erl_nif.h.
#ifdef HAVE_ERL_NIF
#include <erl_nif.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "leoec.h"

namespace {

ERL_NIF_TERM error_tuple(ErlNifEnv* env, const char* why) {
  return enif_make_tuple2(env, enif_make_atom(env, "error"),
                          enif_make_string(env, why, ERL_NIF_LATIN1));
}

// A failure inside the coder (parameter check, block validation, engine).
ERL_NIF_TERM coder_error(ErlNifEnv* env, int rc) {
#ifdef LEOEC_NIF_REF_ERRORS
  (void)rc;
  return error_tuple(env, "std::exception");
#else
  return error_tuple(env, leoec_strerror(rc));
#endif
}

// atom -> CodingType numbering (nif.cpp:61-72); -1 = not a known class
int coding_id(const char* atom) {
  if (!std::strcmp(atom, "cauchyrs")) return LEOEC_CAUCHYRS;
  if (!std::strcmp(atom, "vandrs")) return LEOEC_VANDRS;
  if (!std::strcmp(atom, "liberation")) return LEOEC_LIBERATION;
  if (!std::strcmp(atom, "isars")) return LEOEC_ISARS;
  return -1;
}

// {Class, {K,M,W}} parsing shared by the three NIFs.  Returns nullptr or the
// error message to report.
const char* coding_args(ErlNifEnv* env, ERL_NIF_TERM cls, ERL_NIF_TERM params, int* coding,
                        int* k, int* m, int* w) {
  char atom[64];
  if (!enif_get_atom(env, cls, atom, sizeof atom, ERL_NIF_LATIN1)) return "Expect coding";
  const ERL_NIF_TERM* t;
  int arity;
  if (!enif_get_tuple(env, params, &arity, &t)) return "Expect tuple for coding parameters";
  if (arity < 1 || !enif_get_int(env, t[0], k)) return "Invalid K";
  if (arity < 2 || !enif_get_int(env, t[1], m)) return "Invalid M";
  if (arity < 3 || !enif_get_int(env, t[2], w)) return "Invalid W";
  *coding = coding_id(atom);
  if (*coding < 0) return "Invalid Coding";
  return nullptr;
}

// [Block] + [Id] list parsing (nif.cpp:173-206).
const char* block_lists(ErlNifEnv* env, ERL_NIF_TERM blocks, ERL_NIF_TERM ids,
                        std::vector<ErlNifBinary>* bins, std::vector<int>* idv) {
  unsigned n1, n2;
  if (!enif_get_list_length(env, blocks, &n1)) return "Block List Needed";
  if (!enif_get_list_length(env, ids, &n2)) return "ID List Needed";
  if (n1 != n2) return "Block List and ID List does not match (different Len)";
  bins->resize(n1);
  idv->resize(n1);
  ERL_NIF_TERM bh, bt = blocks, ih, it = ids;
  for (unsigned i = 0; i < n1; ++i) {
    enif_get_list_cell(env, bt, &bh, &bt);
    enif_get_list_cell(env, it, &ih, &it);
    if (!enif_inspect_iolist_as_binary(env, bh, &(*bins)[i])) return "Invalid Block";
    if (!enif_get_int(env, ih, &(*idv)[i])) return "Invalid ID";
  }
  return nullptr;
}

ERL_NIF_TERM nif_gf_init(ErlNifEnv* env, int, const ERL_NIF_TERM[]) {
  const int rc = leoec_gf_init();
#ifdef LEOEC_NIF_REF_ERRORS
  if (rc) return error_tuple(env, "Galois Initialization Failed! w=8");
#endif
  return rc ? coder_error(env, rc) : enif_make_atom(env, "ok");
}

// encode(Class, {K,M,W}, Bin, TotalSize) -> {ok, [Block]} | {error, Reason}
ERL_NIF_TERM nif_encode(ErlNifEnv* env, int, const ERL_NIF_TERM argv[]) {
  ErlNifBinary in;
  ERL_NIF_TERM src = argv[2];
  if (!enif_inspect_binary(env, src, &in)) {  // an iolist: flatten it once
    ErlNifBinary flat, owned;
    if (!enif_inspect_iolist_as_binary(env, src, &flat)) return error_tuple(env, "Expected Input Bin");
    // The flattened bytes are not a binary the NIF owns (enif_make_binary on
    // them would yield no term): copy them into one, so whole data blocks can
    // be sub-binaries of it as for a binary input.
    if (!enif_alloc_binary(flat.size, &owned)) return coder_error(env, LEOEC_E_NOMEM);
    if (flat.size) std::memcpy(owned.data, flat.data, flat.size);
    src = enif_make_binary(env, &owned);
    if (!enif_inspect_binary(env, src, &in)) return coder_error(env, LEOEC_E_NOMEM);
  }
  int coding, k, m, w;
  if (const char* e = coding_args(env, argv[0], argv[1], &coding, &k, &m, &w))
    return error_tuple(env, e);
  uint64_t bs;
  int filled;
  int rc = leoec_layout(coding, k, m, w, in.size, &bs, &filled);
  if (rc) return coder_error(env, rc);
  ErlNifBinary fresh;
  const size_t fresh_size = (size_t)(k + m - filled) * bs;
  if (!enif_alloc_binary(fresh_size, &fresh)) return coder_error(env, LEOEC_E_NOMEM);
  rc = leoec_encode(coding, k, m, w, in.data, in.size, fresh.data, fresh_size);
  if (rc) {
    enif_release_binary(&fresh);
    return coder_error(env, rc);
  }
  std::vector<ERL_NIF_TERM> out;
  out.reserve(k + m);
  for (int i = 0; i < filled; ++i)  // zero-copy, as rscoding.cpp:73-75
    out.push_back(enif_make_sub_binary(env, src, (size_t)i * bs, bs));
  const ERL_NIF_TERM fresh_term = enif_make_binary(env, &fresh);
  for (int i = 0; i < k + m - filled; ++i)
    out.push_back(enif_make_sub_binary(env, fresh_term, (size_t)i * bs, bs));
  return enif_make_tuple2(env, enif_make_atom(env, "ok"),
                          enif_make_list_from_array(env, out.data(), (unsigned)out.size()));
}

// decode(Class, {K,M,W}, [Block], [Id], ObjSize) -> {ok, Bin} | {error, Reason}
ERL_NIF_TERM nif_decode(ErlNifEnv* env, int, const ERL_NIF_TERM argv[]) {
  std::vector<ErlNifBinary> bins;
  std::vector<int> ids;
  if (const char* e = block_lists(env, argv[2], argv[3], &bins, &ids)) return error_tuple(env, e);
  ErlNifUInt64 size;
  if (!enif_get_uint64(env, argv[4], &size)) return error_tuple(env, "Expect data size");
  int coding, k, m, w;
  if (const char* e = coding_args(env, argv[0], argv[1], &coding, &k, &m, &w))
    return error_tuple(env, e);
  const uint64_t bs = bins.empty() ? 0 : bins.back().size;  // rscoding.cpp:102
  std::vector<const uint8_t*> ptrs(bins.size());
  for (size_t i = 0; i < bins.size(); ++i) {
    if (bins[i].size != bs) return coder_error(env, LEOEC_E_BAD_SIZE);
    ptrs[i] = bins[i].data;
  }
  ErlNifBinary out;
  if (!enif_alloc_binary(size, &out)) return coder_error(env, LEOEC_E_NOMEM);
  const int rc = leoec_decode(coding, k, m, w, ptrs.data(), ids.data(), (int)ids.size(), bs, size,
                              out.data);
  if (rc) {
    enif_release_binary(&out);
    return coder_error(env, rc);
  }
  return enif_make_tuple2(env, enif_make_atom(env, "ok"), enif_make_binary(env, &out));
}

// repair(Class, {K,M,W}, [Block], [Id], [RepairId]) -> {ok, [Block]} | {error, Reason}
ERL_NIF_TERM nif_repair(ErlNifEnv* env, int, const ERL_NIF_TERM argv[]) {
  std::vector<ErlNifBinary> bins;
  std::vector<int> ids;
  if (const char* e = block_lists(env, argv[2], argv[3], &bins, &ids)) return error_tuple(env, e);
  unsigned nrep;
  if (!enif_get_list_length(env, argv[4], &nrep)) return error_tuple(env, "Repair ID List Needed");
  std::vector<int> rep(nrep);
  ERL_NIF_TERM h, t = argv[4];
  for (unsigned i = 0; i < nrep; ++i) {
    enif_get_list_cell(env, t, &h, &t);
    if (!enif_get_int(env, h, &rep[i])) return error_tuple(env, "Invalid Repair ID");
  }
  int coding, k, m, w;
  if (const char* e = coding_args(env, argv[0], argv[1], &coding, &k, &m, &w))
    return error_tuple(env, e);
  const uint64_t bs = bins.empty() ? 0 : bins.back().size;
  std::vector<const uint8_t*> ptrs(bins.size());
  for (size_t i = 0; i < bins.size(); ++i) {
    if (bins[i].size != bs) return coder_error(env, LEOEC_E_BAD_SIZE);
    ptrs[i] = bins[i].data;
  }
  ErlNifBinary out;
  if (!enif_alloc_binary((size_t)nrep * bs, &out)) return coder_error(env, LEOEC_E_NOMEM);
  const int rc = leoec_repair(coding, k, m, w, ptrs.data(), ids.data(), (int)ids.size(), bs,
                              rep.data(), (int)nrep, out.data);
  if (rc) {
    enif_release_binary(&out);
    return coder_error(env, rc);
  }
  const ERL_NIF_TERM all = enif_make_binary(env, &out);
  std::vector<ERL_NIF_TERM> blocks(nrep);
  for (unsigned i = 0; i < nrep; ++i) blocks[i] = enif_make_sub_binary(env, all, (size_t)i * bs, bs);
  return enif_make_tuple2(env, enif_make_atom(env, "ok"),
                          enif_make_list_from_array(env, blocks.data(), nrep));
}

ErlNifFunc nif_funcs[] = {
    {"gf_init", 0, nif_gf_init, ERL_NIF_DIRTY_JOB_IO_BOUND},
    {"encode", 4, nif_encode, ERL_NIF_DIRTY_JOB_IO_BOUND},
    {"decode", 5, nif_decode, ERL_NIF_DIRTY_JOB_IO_BOUND},
    {"repair", 5, nif_repair, ERL_NIF_DIRTY_JOB_IO_BOUND},
};

// LEOEC_HOST_DEVICES -> devices; false if malformed.  Unset: "all" (every
// gfx950 device of the process); "" or "current": no spreading (an empty
// set).
bool parse_host_devices(const char* e, std::vector<int>* devs) {
  devs->clear();
  if (!e) e = "all";
  if (!*e || !std::strcmp(e, "current")) return true;
  if (!std::strcmp(e, "all")) {
    const int n = leoec_host_lanes(nullptr, 0);
    if (n > 0) {
      devs->resize((size_t)n);
      if (leoec_host_lanes(devs->data(), n) != n) devs->clear();
    }
    return true;
  }
  for (const char* q = e; *q;) {
    char* end = nullptr;
    const long v = std::strtol(q, &end, 10);
    if (end == q || v < 0 || v > 1023) return false;
    devs->push_back((int)v);
    q = end;
    if (*q == ',') {
      ++q;
      if (!*q) return false;
    } else if (*q) {
      return false;
    }
  }
  return true;
}

int nif_load(ErlNifEnv*, void**, ERL_NIF_TERM) {
  const char* spec = std::getenv("LEOEC_HOST_DEVICES");
  std::vector<int> devs;
  if (!parse_host_devices(spec, &devs)) {
    std::fprintf(stderr, "leo_erasure: malformed LEOEC_HOST_DEVICES=\"%s\"\n", spec);
    return 1;
  }
  if (devs.empty()) return 0;
  const int rc = leoec_host_spread(devs.data(), (int)devs.size());
  if (rc < 0 && leoec_host_lanes(nullptr, 0) > 0) {  // devices exist, the set is not theirs
    std::fprintf(stderr, "leo_erasure: LEOEC_HOST_DEVICES=\"%s\": %s\n", spec ? spec : "(unset: all)",
                 leoec_strerror(rc));
    return 2;
  }
  return 0;
}

}  // namespace

ERL_NIF_INIT(leo_erasure, nif_funcs, nif_load, nullptr, nullptr, nullptr)
#endif  // HAVE_ERL_NIF
