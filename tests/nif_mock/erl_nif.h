/* Stand-in for erts' erl_nif.h (this image has no erts), used two ways:
 *   * tests/test_abi.py type-checks erl/c_src/partisan_gpu_sim_nif.c with
 *     `gcc -fsyntax-only` against these declarations;
 *   * tests/nif_mock/mock_erts.c implements them over a small term arena so
 *     tests/nif_harness.c can link the real NIF shim with libpsim.so and call
 *     its function table as the BEAM would (GPU test, tests/test_nif_harness.py).
 * Signatures follow the documented erl_nif API (erts >= 2.14).  ERL_NIF_INIT
 * here exposes the shim's function table and load callback to the harness. */
#pragma once
#include <stddef.h>
#include <stdint.h>
typedef uint64_t ERL_NIF_TERM;
typedef struct enif_environment_t ErlNifEnv;
typedef struct enif_resource_type_t ErlNifResourceType;
typedef struct ErlNifMutex ErlNifMutex;
typedef unsigned long long ErlNifUInt64;
typedef struct { size_t size; unsigned char* data; void* ref_bin; void* __spare__[2]; } ErlNifBinary;
typedef enum { ERL_NIF_LATIN1 = 1 } ErlNifCharEncoding;
typedef enum { ERL_NIF_RT_CREATE = 1, ERL_NIF_RT_TAKEOVER = 2 } ErlNifResourceFlags;
typedef void ErlNifResourceDtor(ErlNifEnv*, void*);
typedef struct {
    const char* name;
    unsigned arity;
    ERL_NIF_TERM (*fptr)(ErlNifEnv*, int, const ERL_NIF_TERM[]);
    unsigned flags;
} ErlNifFunc;
#define ERL_NIF_DIRTY_JOB_CPU_BOUND 1
int enif_make_existing_atom(ErlNifEnv*, const char*, ERL_NIF_TERM*, ErlNifCharEncoding);
ERL_NIF_TERM enif_make_atom(ErlNifEnv*, const char*);
ERL_NIF_TERM enif_make_tuple2(ErlNifEnv*, ERL_NIF_TERM, ERL_NIF_TERM);
ERL_NIF_TERM enif_make_tuple3(ErlNifEnv*, ERL_NIF_TERM, ERL_NIF_TERM, ERL_NIF_TERM);
ERL_NIF_TERM enif_make_tuple4(ErlNifEnv*, ERL_NIF_TERM, ERL_NIF_TERM, ERL_NIF_TERM, ERL_NIF_TERM);
ERL_NIF_TERM enif_make_tuple5(ErlNifEnv*, ERL_NIF_TERM, ERL_NIF_TERM, ERL_NIF_TERM, ERL_NIF_TERM, ERL_NIF_TERM);
ERL_NIF_TERM enif_make_tuple_from_array(ErlNifEnv*, const ERL_NIF_TERM[], unsigned);
ERL_NIF_TERM enif_make_badarg(ErlNifEnv*);
ERL_NIF_TERM enif_make_uint(ErlNifEnv*, unsigned);
ERL_NIF_TERM enif_make_uint64(ErlNifEnv*, ErlNifUInt64);
ERL_NIF_TERM enif_make_list(ErlNifEnv*, unsigned, ...);
ERL_NIF_TERM enif_make_list_cell(ErlNifEnv*, ERL_NIF_TERM, ERL_NIF_TERM);
ERL_NIF_TERM enif_make_resource(ErlNifEnv*, void*);
unsigned char* enif_make_new_binary(ErlNifEnv*, size_t, ERL_NIF_TERM*);
int enif_make_map_from_arrays(ErlNifEnv*, ERL_NIF_TERM[], ERL_NIF_TERM[], size_t, ERL_NIF_TERM*);
int enif_get_map_value(ErlNifEnv*, ERL_NIF_TERM, ERL_NIF_TERM, ERL_NIF_TERM*);
int enif_is_map(ErlNifEnv*, ERL_NIF_TERM);
int enif_is_identical(ERL_NIF_TERM, ERL_NIF_TERM);
int enif_get_uint(ErlNifEnv*, ERL_NIF_TERM, unsigned*);
int enif_get_uint64(ErlNifEnv*, ERL_NIF_TERM, ErlNifUInt64*);
int enif_inspect_binary(ErlNifEnv*, ERL_NIF_TERM, ErlNifBinary*);
int enif_get_list_cell(ErlNifEnv*, ERL_NIF_TERM, ERL_NIF_TERM*, ERL_NIF_TERM*);
int enif_get_list_length(ErlNifEnv*, ERL_NIF_TERM, unsigned*);
int enif_get_tuple(ErlNifEnv*, ERL_NIF_TERM, int*, const ERL_NIF_TERM**);
ErlNifResourceType* enif_open_resource_type(ErlNifEnv*, const char*, const char*, ErlNifResourceDtor*,
                                            ErlNifResourceFlags, ErlNifResourceFlags*);
void* enif_alloc_resource(ErlNifResourceType*, size_t);
void enif_release_resource(void*);
int enif_get_resource(ErlNifEnv*, ERL_NIF_TERM, ErlNifResourceType*, void**);
void* enif_alloc(size_t);
void enif_free(void*);
ErlNifMutex* enif_mutex_create(char*);
void enif_mutex_destroy(ErlNifMutex*);
void enif_mutex_lock(ErlNifMutex*);
void enif_mutex_unlock(ErlNifMutex*);
typedef int (*mock_nif_load_fn)(ErlNifEnv*, void**, ERL_NIF_TERM);
#define ERL_NIF_INIT(NAME, FUNCS, LOAD, RELOAD, UPGRADE, UNLOAD)                     \
    const ErlNifFunc* mock_nif_table(int* nfuncs_out, mock_nif_load_fn* load_out) {    \
        *nfuncs_out = (int)(sizeof(FUNCS) / sizeof((FUNCS)[0]));                        \
        *load_out = (LOAD);                                                             \
        return (FUNCS);                                                                 \
    }
