/*
 * TEST DOUBLE of the small part of the Erlang NIF API that
 * leo_erasure_amd/csrc/nif/leo_erasure_nif.cpp uses, so that our own NIF
 * shim can be compiled and exercised in this container (Erlang/OTP is not
 * installed).  It is NOT the OTP header and is never used to build the
 * reference: terms are handles into a C++ term store (tests/nif_harness/
 * harness.cpp) driven from pytest.  Semantics follow the erl_nif docs for
 * the calls used: binaries, sub-binaries, atoms, ints, tuples, lists.
 */
#ifndef LEOEC_TEST_ERL_NIF_H
#define LEOEC_TEST_ERL_NIF_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef uintptr_t ERL_NIF_TERM;
typedef uint64_t ErlNifUInt64;
typedef struct enif_environment_t ErlNifEnv;

typedef struct {
  size_t size;
  unsigned char *data;
  void *ref_bin; /* owner handle (harness internal) */
} ErlNifBinary;

typedef enum { ERL_NIF_LATIN1 = 1 } ErlNifCharEncoding;

#define ERL_NIF_DIRTY_JOB_CPU_BOUND 1
#define ERL_NIF_DIRTY_JOB_IO_BOUND 2

typedef struct {
  const char *name;
  unsigned arity;
  ERL_NIF_TERM (*fptr)(ErlNifEnv *env, int argc, const ERL_NIF_TERM argv[]);
  unsigned flags;
} ErlNifFunc;

ERL_NIF_TERM enif_make_atom(ErlNifEnv *env, const char *name);
ERL_NIF_TERM enif_make_string(ErlNifEnv *env, const char *s, ErlNifCharEncoding enc);
ERL_NIF_TERM enif_make_tuple2(ErlNifEnv *env, ERL_NIF_TERM a, ERL_NIF_TERM b);
ERL_NIF_TERM enif_make_binary(ErlNifEnv *env, ErlNifBinary *bin);
ERL_NIF_TERM enif_make_sub_binary(ErlNifEnv *env, ERL_NIF_TERM bin, size_t pos, size_t size);
ERL_NIF_TERM enif_make_list_from_array(ErlNifEnv *env, const ERL_NIF_TERM arr[], unsigned cnt);
int enif_get_atom(ErlNifEnv *env, ERL_NIF_TERM t, char *buf, unsigned len, ErlNifCharEncoding enc);
int enif_get_tuple(ErlNifEnv *env, ERL_NIF_TERM t, int *arity, const ERL_NIF_TERM **array);
int enif_get_int(ErlNifEnv *env, ERL_NIF_TERM t, int *ip);
int enif_get_uint64(ErlNifEnv *env, ERL_NIF_TERM t, ErlNifUInt64 *ip);
int enif_get_list_length(ErlNifEnv *env, ERL_NIF_TERM t, unsigned *len);
int enif_get_list_cell(ErlNifEnv *env, ERL_NIF_TERM list, ERL_NIF_TERM *head, ERL_NIF_TERM *tail);
int enif_inspect_binary(ErlNifEnv *env, ERL_NIF_TERM t, ErlNifBinary *bin);
int enif_inspect_iolist_as_binary(ErlNifEnv *env, ERL_NIF_TERM t, ErlNifBinary *bin);
int enif_alloc_binary(size_t size, ErlNifBinary *bin);
void enif_release_binary(ErlNifBinary *bin);

/* The shim's ERL_NIF_INIT(leo_erasure, funcs, load, ...) exposes its table
 * and its load callback (called as the VM would, load_info 0) here. */
const ErlNifFunc *leoec_test_nif_table(unsigned *count);
int leoec_test_nif_load(void);
#define ERL_NIF_INIT(MOD, FUNCS, LOAD, RELOAD, UPGRADE, UNLOAD)                 \
  extern "C" const ErlNifFunc *leoec_test_nif_table(unsigned *count) {         \
    *count = (unsigned)(sizeof(FUNCS) / sizeof(FUNCS[0]));                     \
    return FUNCS;                                                              \
  }                                                                            \
  extern "C" int leoec_test_nif_load(void) {                                   \
    int (*f)(ErlNifEnv *, void **, ERL_NIF_TERM) = LOAD;                       \
    return f ? f(nullptr, nullptr, 0) : 0;                                     \
  }

#ifdef __cplusplus
}
#endif
#endif
