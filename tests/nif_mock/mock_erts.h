/* mock_erts.h -- harness-side helpers of tests/nif_mock/mock_erts.c (test
 * infrastructure: builds and reads terms of the mock term store). */
#pragma once
#include "erl_nif.h"

ERL_NIF_TERM mock_atom(const char* name);
ERL_NIF_TERM mock_uint(uint64_t v);
ERL_NIF_TERM mock_bin(const void* data, size_t size);
ERL_NIF_TERM mock_map(size_t n, const char* const* keys, const uint64_t* vals);
int mock_is_atom(ERL_NIF_TERM t, const char* name);
int mock_is_badarg(ERL_NIF_TERM t);
size_t mock_tuple_arity(ERL_NIF_TERM t);
ERL_NIF_TERM mock_elem(ERL_NIF_TERM t, size_t i);
uint64_t mock_int(ERL_NIF_TERM t);
const unsigned char* mock_bin_data(ERL_NIF_TERM t, size_t* size);
size_t mock_list_len(ERL_NIF_TERM t);
ERL_NIF_TERM mock_list_nth(ERL_NIF_TERM t, size_t i);
int mock_map_get(ERL_NIF_TERM map, const char* key, uint64_t* out);
const char* mock_atom_name(ERL_NIF_TERM t);
void mock_drop_terms(void);   /* drop every term's resource reference (runs destructors) */
/* the shim's table (ERL_NIF_INIT in erl_nif.h) */
const ErlNifFunc* mock_nif_table(int* n, mock_nif_load_fn* load);
