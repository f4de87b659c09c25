/*
 * build_tree.c -- restatement of partisan_plumtree_util:build_tree/3
 * (src/partisan_plumtree_util.erl:43-58).  TEST INFRASTRUCTURE ONLY.
 *
 * Expand = cycles ? Nodes repeated N+1 times : Nodes; fold over Nodes taking
 * min(N, length(Worklist)) children off tl(Expand); result as an orddict
 * (sorted by node; node ids given here sort like the atoms node1..nodeK).
 */
#include "oracle.h"
#include <stdlib.h>
#include <string.h>

int orc_build_tree(uint32_t arity, const uint32_t* nodes, size_t n, int cycles,
                   uint32_t* out_keys, uint32_t* out_children, uint32_t* out_counts) {
    if (n == 0) return ORC_OK;
    size_t nexp = cycles ? n * (arity + 1) : n;
    uint32_t* expand = (uint32_t*)malloc(nexp * sizeof(uint32_t));
    for (size_t i = 0; i < nexp; i++) expand[i] = nodes[i % n];
    size_t wl = 1;                                   /* Worklist = tl(Expand) */
    uint32_t* keys = (uint32_t*)malloc(n * sizeof(uint32_t));
    uint32_t* ch = (uint32_t*)malloc(n * arity * sizeof(uint32_t) + 4);
    uint32_t* cnt = (uint32_t*)malloc(n * sizeof(uint32_t));
    for (size_t i = 0; i < n; i++) {
        size_t remaining = nexp - wl;
        size_t len = arity < remaining ? arity : remaining;
        keys[i] = nodes[i];
        for (size_t j = 0; j < len; j++) ch[i * arity + j] = expand[wl + j];
        cnt[i] = (uint32_t)len;
        wl += len;
    }
    /* orddict:from_list: sort by key; a later duplicate key replaces an earlier one */
    size_t* idx = (size_t*)malloc(n * sizeof(size_t));
    for (size_t i = 0; i < n; i++) idx[i] = i;
    for (size_t i = 1; i < n; i++) {
        size_t x = idx[i], j = i;
        while (j > 0 && keys[idx[j - 1]] > keys[x]) { idx[j] = idx[j - 1]; j--; }
        idx[j] = x;
    }
    for (size_t i = 0; i < n; i++) {
        size_t s = idx[i];
        out_keys[i] = keys[s];
        out_counts[i] = cnt[s];
        memcpy(&out_children[i * arity], &ch[s * arity], cnt[s] * sizeof(uint32_t));
    }
    free(expand); free(keys); free(ch); free(cnt); free(idx);
    return ORC_OK;
}
