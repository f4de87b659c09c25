/* mock_erts.c -- a minimal term store implementing the erl_nif calls that
 * erl/c_src/partisan_gpu_sim_nif.c makes, so the real NIF shim can be linked
 * with libpsim.so and driven by tests/nif_harness.c in an image without erts.
 * TEST INFRASTRUCTURE: terms live in one growing arena (never collected);
 * resources are reference counted as in erts (make_resource takes a
 * reference, release_resource drops the creator's; mock_drop_terms() drops
 * the terms' references, running the destructors). */
#include "mock_erts.h"

#include <pthread.h>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

typedef enum { T_NIL, T_ATOM, T_INT, T_BIN, T_TUPLE, T_CONS, T_MAP, T_RES, T_BADARG } tag_t;

typedef struct {
    tag_t tag;
    uint64_t u;            /* atom id / integer */
    size_t n;              /* binary size / tuple arity / map size */
    unsigned char* bin;
    ERL_NIF_TERM* a;       /* tuple items / map keys / cons {head, tail} */
    ERL_NIF_TERM* b;       /* map values */
    void* res;
} term_t;

struct enif_resource_type_t {
    ErlNifResourceDtor* dtor;
};

typedef struct {
    ErlNifResourceType* type;
    int refc;
    double align_;          /* payload alignment */
} res_hdr;

static term_t* arena;
static size_t n_terms, cap_terms;
static char** atoms;
static size_t n_atoms, cap_atoms;
static ERL_NIF_TERM* atom_term;

static ERL_NIF_TERM push(term_t t) {
    if (n_terms == cap_terms) {
        cap_terms = cap_terms ? 2 * cap_terms : 4096;
        arena = (term_t*)realloc(arena, cap_terms * sizeof(term_t));
        if (!arena) abort();
    }
    arena[n_terms] = t;
    return (ERL_NIF_TERM)n_terms++;
}

static term_t* T(ERL_NIF_TERM t) {
    if (t >= n_terms) {
        fprintf(stderr, "mock_erts: bad term %llu\n", (unsigned long long)t);
        abort();
    }
    return &arena[t];
}

/* ---- erl_nif API --------------------------------------------------------- */
int enif_make_existing_atom(ErlNifEnv* env, const char* name, ERL_NIF_TERM* out, ErlNifCharEncoding enc) {
    (void)env;
    (void)enc;
    for (size_t i = 0; i < n_atoms; i++)
        if (!strcmp(atoms[i], name)) {
            *out = atom_term[i];
            return 1;
        }
    return 0;
}

ERL_NIF_TERM enif_make_atom(ErlNifEnv* env, const char* name) {
    ERL_NIF_TERM t;
    if (enif_make_existing_atom(env, name, &t, ERL_NIF_LATIN1)) return t;
    if (n_atoms == cap_atoms) {
        cap_atoms = cap_atoms ? 2 * cap_atoms : 64;
        atoms = (char**)realloc(atoms, cap_atoms * sizeof(char*));
        atom_term = (ERL_NIF_TERM*)realloc(atom_term, cap_atoms * sizeof(ERL_NIF_TERM));
    }
    term_t x = {0};
    x.tag = T_ATOM;
    x.u = n_atoms;
    atoms[n_atoms] = strdup(name);
    atom_term[n_atoms] = push(x);
    return atom_term[n_atoms++];
}

ERL_NIF_TERM enif_make_tuple_from_array(ErlNifEnv* env, const ERL_NIF_TERM items[], unsigned n) {
    (void)env;
    term_t x = {0};
    x.tag = T_TUPLE;
    x.n = n;
    x.a = (ERL_NIF_TERM*)malloc((n ? n : 1) * sizeof(ERL_NIF_TERM));
    memcpy(x.a, items, n * sizeof(ERL_NIF_TERM));
    return push(x);
}
ERL_NIF_TERM enif_make_tuple2(ErlNifEnv* e, ERL_NIF_TERM a, ERL_NIF_TERM b) {
    ERL_NIF_TERM v[2] = {a, b};
    return enif_make_tuple_from_array(e, v, 2);
}
ERL_NIF_TERM enif_make_tuple3(ErlNifEnv* e, ERL_NIF_TERM a, ERL_NIF_TERM b, ERL_NIF_TERM c) {
    ERL_NIF_TERM v[3] = {a, b, c};
    return enif_make_tuple_from_array(e, v, 3);
}
ERL_NIF_TERM enif_make_tuple4(ErlNifEnv* e, ERL_NIF_TERM a, ERL_NIF_TERM b, ERL_NIF_TERM c, ERL_NIF_TERM d) {
    ERL_NIF_TERM v[4] = {a, b, c, d};
    return enif_make_tuple_from_array(e, v, 4);
}
ERL_NIF_TERM enif_make_tuple5(ErlNifEnv* e, ERL_NIF_TERM a, ERL_NIF_TERM b, ERL_NIF_TERM c, ERL_NIF_TERM d,
                              ERL_NIF_TERM f) {
    ERL_NIF_TERM v[5] = {a, b, c, d, f};
    return enif_make_tuple_from_array(e, v, 5);
}

ERL_NIF_TERM enif_make_badarg(ErlNifEnv* env) {
    (void)env;
    term_t x = {0};
    x.tag = T_BADARG;
    return push(x);
}

ERL_NIF_TERM enif_make_uint64(ErlNifEnv* env, ErlNifUInt64 v) {
    (void)env;
    term_t x = {0};
    x.tag = T_INT;
    x.u = v;
    return push(x);
}
ERL_NIF_TERM enif_make_uint(ErlNifEnv* env, unsigned v) { return enif_make_uint64(env, v); }

ERL_NIF_TERM enif_make_list(ErlNifEnv* env, unsigned n, ...) {
    (void)env;
    if (n != 0) {
        fprintf(stderr, "mock_erts: enif_make_list with elements is not modelled\n");
        abort();
    }
    term_t x = {0};
    x.tag = T_NIL;
    return push(x);
}

ERL_NIF_TERM enif_make_list_cell(ErlNifEnv* env, ERL_NIF_TERM head, ERL_NIF_TERM tail) {
    (void)env;
    term_t x = {0};
    x.tag = T_CONS;
    x.a = (ERL_NIF_TERM*)malloc(2 * sizeof(ERL_NIF_TERM));
    x.a[0] = head;
    x.a[1] = tail;
    return push(x);
}

ERL_NIF_TERM enif_make_resource(ErlNifEnv* env, void* obj) {
    (void)env;
    res_hdr* h = (res_hdr*)obj - 1;
    h->refc++;
    term_t x = {0};
    x.tag = T_RES;
    x.res = obj;
    return push(x);
}

unsigned char* enif_make_new_binary(ErlNifEnv* env, size_t size, ERL_NIF_TERM* out) {
    (void)env;
    term_t x = {0};
    x.tag = T_BIN;
    x.n = size;
    x.bin = (unsigned char*)calloc(size ? size : 1, 1);
    *out = push(x);
    return x.bin;
}

int enif_make_map_from_arrays(ErlNifEnv* env, ERL_NIF_TERM keys[], ERL_NIF_TERM vals[], size_t n, ERL_NIF_TERM* out) {
    (void)env;
    term_t x = {0};
    x.tag = T_MAP;
    x.n = n;
    x.a = (ERL_NIF_TERM*)malloc((n ? n : 1) * sizeof(ERL_NIF_TERM));
    x.b = (ERL_NIF_TERM*)malloc((n ? n : 1) * sizeof(ERL_NIF_TERM));
    memcpy(x.a, keys, n * sizeof(ERL_NIF_TERM));
    memcpy(x.b, vals, n * sizeof(ERL_NIF_TERM));
    *out = push(x);
    return 1;
}

int enif_is_identical(ERL_NIF_TERM a, ERL_NIF_TERM b) {
    if (a == b) return 1;
    term_t *x = T(a), *y = T(b);
    if (x->tag != y->tag) return 0;
    switch (x->tag) {
    case T_NIL: return 1;
    case T_ATOM:
    case T_INT: return x->u == y->u;
    case T_BIN: return x->n == y->n && !memcmp(x->bin, y->bin, x->n);
    case T_RES: return x->res == y->res;
    case T_TUPLE:
        if (x->n != y->n) return 0;
        for (size_t i = 0; i < x->n; i++)
            if (!enif_is_identical(x->a[i], y->a[i])) return 0;
        return 1;
    case T_CONS: return enif_is_identical(x->a[0], y->a[0]) && enif_is_identical(x->a[1], y->a[1]);
    default: return 0;
    }
}

int enif_get_map_value(ErlNifEnv* env, ERL_NIF_TERM map, ERL_NIF_TERM key, ERL_NIF_TERM* val) {
    (void)env;
    term_t* m = T(map);
    if (m->tag != T_MAP) return 0;
    for (size_t i = 0; i < m->n; i++)
        if (enif_is_identical(m->a[i], key)) {
            *val = m->b[i];
            return 1;
        }
    return 0;
}

int enif_is_map(ErlNifEnv* env, ERL_NIF_TERM t) {
    (void)env;
    return T(t)->tag == T_MAP;
}

int enif_get_uint64(ErlNifEnv* env, ERL_NIF_TERM t, ErlNifUInt64* out) {
    (void)env;
    if (T(t)->tag != T_INT) return 0;
    *out = T(t)->u;
    return 1;
}

int enif_get_uint(ErlNifEnv* env, ERL_NIF_TERM t, unsigned* out) {
    ErlNifUInt64 v;
    if (!enif_get_uint64(env, t, &v) || v > 0xFFFFFFFFull) return 0;
    *out = (unsigned)v;
    return 1;
}

int enif_get_list_cell(ErlNifEnv* env, ERL_NIF_TERM list, ERL_NIF_TERM* head, ERL_NIF_TERM* tail) {
    (void)env;
    term_t* x = T(list);
    if (x->tag != T_CONS) return 0;
    *head = x->a[0];
    *tail = x->a[1];
    return 1;
}

int enif_get_list_length(ErlNifEnv* env, ERL_NIF_TERM list, unsigned* len) {
    (void)env;
    unsigned n = 0;
    while (T(list)->tag == T_CONS) {
        n++;
        list = T(list)->a[1];
    }
    if (T(list)->tag != T_NIL) return 0;
    *len = n;
    return 1;
}

int enif_get_tuple(ErlNifEnv* env, ERL_NIF_TERM t, int* arity, const ERL_NIF_TERM** items) {
    (void)env;
    term_t* x = T(t);
    if (x->tag != T_TUPLE) return 0;
    *arity = (int)x->n;
    *items = x->a;
    return 1;
}

int enif_inspect_binary(ErlNifEnv* env, ERL_NIF_TERM t, ErlNifBinary* bin) {
    (void)env;
    term_t* x = T(t);
    if (x->tag != T_BIN) return 0;
    memset(bin, 0, sizeof *bin);
    bin->size = x->n;
    bin->data = x->bin;
    return 1;
}

ErlNifResourceType* enif_open_resource_type(ErlNifEnv* env, const char* mod, const char* name,
                                            ErlNifResourceDtor* dtor, ErlNifResourceFlags flags,
                                            ErlNifResourceFlags* tried) {
    (void)env;
    (void)mod;
    (void)name;
    (void)flags;
    (void)tried;
    ErlNifResourceType* t = (ErlNifResourceType*)calloc(1, sizeof *t);
    t->dtor = dtor;
    return t;
}

void* enif_alloc_resource(ErlNifResourceType* type, size_t size) {
    res_hdr* h = (res_hdr*)calloc(1, sizeof(res_hdr) + size);
    h->type = type;
    h->refc = 1;
    return h + 1;
}

void enif_release_resource(void* obj) {
    res_hdr* h = (res_hdr*)obj - 1;
    if (--h->refc == 0) {
        if (h->type->dtor) h->type->dtor(NULL, obj);
        free(h);
    }
}

int enif_get_resource(ErlNifEnv* env, ERL_NIF_TERM t, ErlNifResourceType* type, void** obj) {
    (void)env;
    term_t* x = T(t);
    if (x->tag != T_RES || ((res_hdr*)x->res - 1)->type != type) return 0;
    *obj = x->res;
    return 1;
}

void* enif_alloc(size_t n) { return malloc(n ? n : 1); }
void enif_free(void* p) { free(p); }

struct ErlNifMutex {
    pthread_mutex_t m;
};
ErlNifMutex* enif_mutex_create(char* name) {
    (void)name;
    ErlNifMutex* m = (ErlNifMutex*)calloc(1, sizeof *m);
    pthread_mutex_init(&m->m, NULL);
    return m;
}
void enif_mutex_destroy(ErlNifMutex* m) {
    pthread_mutex_destroy(&m->m);
    free(m);
}
void enif_mutex_lock(ErlNifMutex* m) { pthread_mutex_lock(&m->m); }
void enif_mutex_unlock(ErlNifMutex* m) { pthread_mutex_unlock(&m->m); }

/* ---- harness helpers ------------------------------------------------------ */
ERL_NIF_TERM mock_atom(const char* name) { return enif_make_atom(NULL, name); }
ERL_NIF_TERM mock_uint(uint64_t v) { return enif_make_uint64(NULL, v); }
ERL_NIF_TERM mock_bin(const void* data, size_t size) {
    ERL_NIF_TERM t;
    unsigned char* p = enif_make_new_binary(NULL, size, &t);
    if (size) memcpy(p, data, size);
    return t;
}
ERL_NIF_TERM mock_map(size_t n, const char* const* keys, const uint64_t* vals) {
    ERL_NIF_TERM k[32], v[32], m;
    for (size_t i = 0; i < n && i < 32; i++) {
        k[i] = mock_atom(keys[i]);
        v[i] = mock_uint(vals[i]);
    }
    enif_make_map_from_arrays(NULL, k, v, n, &m);
    return m;
}
int mock_is_atom(ERL_NIF_TERM t, const char* name) {
    ERL_NIF_TERM a;
    return T(t)->tag == T_ATOM && enif_make_existing_atom(NULL, name, &a, ERL_NIF_LATIN1) && a == t;
}
int mock_is_badarg(ERL_NIF_TERM t) { return T(t)->tag == T_BADARG; }
size_t mock_tuple_arity(ERL_NIF_TERM t) { return T(t)->tag == T_TUPLE ? T(t)->n : 0; }
ERL_NIF_TERM mock_elem(ERL_NIF_TERM t, size_t i) {
    if (T(t)->tag != T_TUPLE || i >= T(t)->n) abort();
    return T(t)->a[i];
}
uint64_t mock_int(ERL_NIF_TERM t) {
    if (T(t)->tag != T_INT) abort();
    return T(t)->u;
}
const unsigned char* mock_bin_data(ERL_NIF_TERM t, size_t* size) {
    if (T(t)->tag != T_BIN) abort();
    *size = T(t)->n;
    return T(t)->bin;
}
size_t mock_list_len(ERL_NIF_TERM t) {
    size_t n = 0;
    while (T(t)->tag == T_CONS) {
        n++;
        t = T(t)->a[1];
    }
    return n;
}
ERL_NIF_TERM mock_list_nth(ERL_NIF_TERM t, size_t i) {
    while (i--) t = T(t)->a[1];
    if (T(t)->tag != T_CONS) abort();
    return T(t)->a[0];
}
int mock_map_get(ERL_NIF_TERM map, const char* key, uint64_t* out) {
    ERL_NIF_TERM v;
    if (!enif_get_map_value(NULL, map, mock_atom(key), &v)) return 0;
    *out = mock_int(v);
    return 1;
}
const char* mock_atom_name(ERL_NIF_TERM t) { return T(t)->tag == T_ATOM ? atoms[T(t)->u] : NULL; }
void mock_drop_terms(void) {
    for (size_t i = 0; i < n_terms; i++)
        if (arena[i].tag == T_RES && arena[i].res) {
            void* obj = arena[i].res;
            arena[i].res = NULL;
            enif_release_resource(obj);
        }
}
