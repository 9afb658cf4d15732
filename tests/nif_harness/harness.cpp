// TEST DOUBLE term store behind tests/nif_harness/erl_nif.h.
//
// Lets pytest drive our own NIF shim (leo_erasure_amd/csrc/nif/
// leo_erasure_nif.cpp) without an Erlang VM: terms are indices into a
// process-wide store, binaries are reference-counted owners so that
// sub-binaries alias their parent (the zero-copy behaviour the shim relies on
// for data blocks, cf. reference c_src/rscoding.cpp:73-75), and the h_* entry
// points below are what tests/test_nif_shim.py binds with ctypes.  Not part
// of the product; never linked into libleoec.so.
#include "erl_nif.h"

#include <climits>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <string>
#include <vector>

namespace {

struct Owner {
  std::vector<unsigned char> bytes;
  long id;
};

enum Kind { ATOM = 0, INT = 1, BIN = 2, TUPLE = 3, LIST = 4 };

struct Term {
  Kind kind;
  long long ival = 0;
  std::string atom;
  std::shared_ptr<Owner> owner;  // BIN
  size_t off = 0, size = 0;      // BIN view into owner
  std::shared_ptr<std::vector<ERL_NIF_TERM>> elems;  // TUPLE / LIST
  size_t start = 0;              // LIST: cons cell = elems[start..]
};

std::vector<Term> g_terms;  // handle = index + 1
long g_next_owner = 1;
long g_live_allocs = 0;     // enif_alloc_binary'd, neither made into a term nor released
long g_violations = 0;      // out-of-range sub-binary etc.

ERL_NIF_TERM put(Term t) {
  g_terms.push_back(std::move(t));
  return (ERL_NIF_TERM)g_terms.size();
}
Term* get(ERL_NIF_TERM h) {
  if (h == 0 || h > g_terms.size()) return nullptr;
  return &g_terms[h - 1];
}
std::shared_ptr<Owner> new_owner(size_t n) {
  auto o = std::make_shared<Owner>();
  o->bytes.resize(n);
  o->id = g_next_owner++;
  return o;
}
// Binaries handed out by enif_alloc_binary, keyed by ErlNifBinary::ref_bin.
std::vector<std::shared_ptr<Owner>> g_pending;

ERL_NIF_TERM make_list(const ERL_NIF_TERM* a, size_t n) {
  Term t;
  t.kind = LIST;
  t.elems = std::make_shared<std::vector<ERL_NIF_TERM>>(a, a + n);
  return put(std::move(t));
}

bool flatten(ERL_NIF_TERM h, std::vector<unsigned char>* out, int depth) {
  Term* t = get(h);
  if (!t || depth > 100) return false;
  if (t->kind == BIN) {
    const unsigned char* p = t->owner->bytes.data() + t->off;
    out->insert(out->end(), p, p + t->size);
    return true;
  }
  if (t->kind != LIST) return false;
  auto elems = t->elems;
  for (size_t i = t->start; i < elems->size(); ++i) {
    Term* e = get((*elems)[i]);
    if (!e) return false;
    if (e->kind == INT) {
      if (e->ival < 0 || e->ival > 255) return false;
      out->push_back((unsigned char)e->ival);
    } else if (!flatten((*elems)[i], out, depth + 1)) {
      return false;
    }
  }
  return true;
}

}  // namespace

extern "C" {

// ---- erl_nif API subset --------------------------------------------------
ERL_NIF_TERM enif_make_atom(ErlNifEnv*, const char* name) {
  Term t;
  t.kind = ATOM;
  t.atom = name;
  return put(std::move(t));
}

ERL_NIF_TERM enif_make_string(ErlNifEnv*, const char* s, ErlNifCharEncoding) {
  std::vector<ERL_NIF_TERM> cs;
  for (const unsigned char* p = (const unsigned char*)s; *p; ++p) {
    Term c;
    c.kind = INT;
    c.ival = *p;
    cs.push_back(put(std::move(c)));
  }
  return make_list(cs.data(), cs.size());
}

ERL_NIF_TERM enif_make_tuple2(ErlNifEnv*, ERL_NIF_TERM a, ERL_NIF_TERM b) {
  Term t;
  t.kind = TUPLE;
  t.elems = std::make_shared<std::vector<ERL_NIF_TERM>>(std::vector<ERL_NIF_TERM>{a, b});
  return put(std::move(t));
}

ERL_NIF_TERM enif_make_binary(ErlNifEnv*, ErlNifBinary* bin) {
  Term t;
  t.kind = BIN;
  t.size = bin->size;
  for (size_t i = 0; i < g_pending.size(); ++i) {
    if (g_pending[i].get() == bin->ref_bin) {  // ownership moves to the term
      t.owner = g_pending[i];
      g_pending.erase(g_pending.begin() + i);
      --g_live_allocs;
      return put(std::move(t));
    }
  }
  // Not an enif_alloc_binary'd buffer (e.g. the result of
  // enif_inspect_iolist_as_binary): real ERTS returns THE_NON_VALUE here,
  // which crashes the VM once used as a term.  Count it and hand back the
  // invalid handle 0.
  ++g_violations;
  return 0;
}

ERL_NIF_TERM enif_make_sub_binary(ErlNifEnv*, ERL_NIF_TERM bin, size_t pos, size_t size) {
  Term* b = get(bin);
  if (!b || b->kind != BIN || pos > b->size || size > b->size - pos) {
    ++g_violations;
    return 0;
  }
  Term t;
  t.kind = BIN;
  t.owner = b->owner;
  t.off = b->off + pos;
  t.size = size;
  return put(std::move(t));
}

ERL_NIF_TERM enif_make_list_from_array(ErlNifEnv*, const ERL_NIF_TERM arr[], unsigned cnt) {
  return make_list(arr, cnt);
}

int enif_get_atom(ErlNifEnv*, ERL_NIF_TERM h, char* buf, unsigned len, ErlNifCharEncoding) {
  Term* t = get(h);
  if (!t || t->kind != ATOM || t->atom.size() + 1 > len) return 0;
  std::memcpy(buf, t->atom.c_str(), t->atom.size() + 1);
  return (int)t->atom.size() + 1;
}

int enif_get_tuple(ErlNifEnv*, ERL_NIF_TERM h, int* arity, const ERL_NIF_TERM** array) {
  Term* t = get(h);
  if (!t || t->kind != TUPLE) return 0;
  *arity = (int)t->elems->size();
  *array = t->elems->data();
  return 1;
}

int enif_get_int(ErlNifEnv*, ERL_NIF_TERM h, int* ip) {
  Term* t = get(h);
  if (!t || t->kind != INT || t->ival < INT_MIN || t->ival > INT_MAX) return 0;
  *ip = (int)t->ival;
  return 1;
}

int enif_get_uint64(ErlNifEnv*, ERL_NIF_TERM h, ErlNifUInt64* ip) {
  Term* t = get(h);
  if (!t || t->kind != INT || t->ival < 0) return 0;
  *ip = (ErlNifUInt64)t->ival;
  return 1;
}

int enif_get_list_length(ErlNifEnv*, ERL_NIF_TERM h, unsigned* len) {
  Term* t = get(h);
  if (!t || t->kind != LIST) return 0;
  *len = (unsigned)(t->elems->size() - t->start);
  return 1;
}

int enif_get_list_cell(ErlNifEnv*, ERL_NIF_TERM h, ERL_NIF_TERM* head, ERL_NIF_TERM* tail) {
  Term* t = get(h);
  if (!t || t->kind != LIST || t->start >= t->elems->size()) return 0;
  *head = (*t->elems)[t->start];
  Term rest;
  rest.kind = LIST;
  rest.elems = t->elems;
  rest.start = t->start + 1;
  *tail = put(std::move(rest));  // may reallocate g_terms: t is dead past here
  return 1;
}

int enif_inspect_binary(ErlNifEnv*, ERL_NIF_TERM h, ErlNifBinary* bin) {
  Term* t = get(h);
  if (!t || t->kind != BIN) return 0;
  bin->size = t->size;
  bin->data = t->owner->bytes.data() + t->off;
  bin->ref_bin = nullptr;
  return 1;
}

int enif_inspect_iolist_as_binary(ErlNifEnv* env, ERL_NIF_TERM h, ErlNifBinary* bin) {
  Term* t = get(h);
  if (!t) return 0;
  if (t->kind == BIN) return enif_inspect_binary(env, h, bin);
  std::vector<unsigned char> flat;
  if (!flatten(h, &flat, 0)) return 0;
  // The VM keeps the flattened copy alive for the NIF call; park it in a term.
  Term keep;
  keep.kind = BIN;
  keep.owner = new_owner(flat.size());
  if (!flat.empty()) std::memcpy(keep.owner->bytes.data(), flat.data(), flat.size());
  keep.size = flat.size();
  const ERL_NIF_TERM k = put(std::move(keep));
  return enif_inspect_binary(env, k, bin);
}

int enif_alloc_binary(size_t size, ErlNifBinary* bin) {
  auto o = new_owner(size);
  g_pending.push_back(o);
  ++g_live_allocs;
  bin->size = size;
  bin->data = o->bytes.data();
  bin->ref_bin = o.get();
  return 1;
}

void enif_release_binary(ErlNifBinary* bin) {
  for (size_t i = 0; i < g_pending.size(); ++i) {
    if (g_pending[i].get() == bin->ref_bin) {
      g_pending.erase(g_pending.begin() + i);
      --g_live_allocs;
      return;
    }
  }
  ++g_violations;  // releasing something that was not allocated / already consumed
}

// ---- harness entry points (ctypes) ---------------------------------------
void h_reset(void) {
  g_terms.clear();
  g_pending.clear();
  g_live_allocs = 0;
  g_violations = 0;
}
long h_live_allocs(void) { return g_live_allocs; }
long h_violations(void) { return g_violations; }

ERL_NIF_TERM h_atom(const char* s) { return enif_make_atom(nullptr, s); }
ERL_NIF_TERM h_int(long long v) {
  Term t;
  t.kind = INT;
  t.ival = v;
  return put(std::move(t));
}
ERL_NIF_TERM h_bin(const unsigned char* p, size_t n) {
  Term t;
  t.kind = BIN;
  t.owner = new_owner(n);
  if (n) std::memcpy(t.owner->bytes.data(), p, n);
  t.size = n;
  return put(std::move(t));
}
ERL_NIF_TERM h_sub(ERL_NIF_TERM bin, size_t pos, size_t n) {
  return enif_make_sub_binary(nullptr, bin, pos, n);
}
ERL_NIF_TERM h_tuple(const ERL_NIF_TERM* a, unsigned n) {
  Term t;
  t.kind = TUPLE;
  t.elems = std::make_shared<std::vector<ERL_NIF_TERM>>(a, a + n);
  return put(std::move(t));
}
ERL_NIF_TERM h_list(const ERL_NIF_TERM* a, unsigned n) { return make_list(a, n); }

int h_kind(ERL_NIF_TERM h) {
  Term* t = get(h);
  return t ? (int)t->kind : -1;
}
long long h_intval(ERL_NIF_TERM h) { return get(h)->ival; }
const char* h_atomname(ERL_NIF_TERM h) { return get(h)->atom.c_str(); }
unsigned h_len(ERL_NIF_TERM h) {
  Term* t = get(h);
  return (unsigned)(t->kind == BIN ? t->size : t->elems->size() - t->start);
}
ERL_NIF_TERM h_elem(ERL_NIF_TERM h, unsigned i) {
  Term* t = get(h);
  return (*t->elems)[t->start + i];
}
const unsigned char* h_bindata(ERL_NIF_TERM h) {
  Term* t = get(h);
  return t->owner->bytes.data() + t->off;
}
long h_binowner(ERL_NIF_TERM h) { return get(h)->owner->id; }
size_t h_binoff(ERL_NIF_TERM h) { return get(h)->off; }

// Look the NIF up in the shim's ErlNifFunc table by name and arity.
ERL_NIF_TERM h_call(const char* name, int argc, const ERL_NIF_TERM* argv, unsigned* flags) {
  unsigned n = 0;
  const ErlNifFunc* f = leoec_test_nif_table(&n);
  for (unsigned i = 0; i < n; ++i) {
    if (!std::strcmp(f[i].name, name) && (int)f[i].arity == argc) {
      if (flags) *flags = f[i].flags;
      return f[i].fptr(nullptr, argc, argv);
    }
  }
  return 0;
}
int h_load(void) { return leoec_test_nif_load(); }
unsigned h_nfuncs(void) {
  unsigned n = 0;
  leoec_test_nif_table(&n);
  return n;
}
const char* h_func(unsigned i, unsigned* arity, unsigned* flags) {
  unsigned n = 0;
  const ErlNifFunc* f = leoec_test_nif_table(&n);
  *arity = f[i].arity;
  *flags = f[i].flags;
  return f[i].name;
}

}  // extern "C"
