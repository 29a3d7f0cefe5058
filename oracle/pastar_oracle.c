/*
 * pastar_oracle.c -- CPU restatement of the reference PAStar hot path
 * (Gabrielcarvfer/mpi_pastar_msa, paths below relative to its root).
 *
 * TEST INFRASTRUCTURE ONLY (see pastar_oracle.h).  Plain C, no dependencies.
 * Compile with -ffp-contract=off and without fast-math: the Altschul weight
 * pipeline is IEEE single arithmetic whose (int) truncation must match the
 * reference bit for bit (SURVEY.md §7 hard part (a)).
 *
 * Parity pinning.  The reference has no tests and no golden files (SURVEY.md
 * §4) and as a whole is unbuildable here (Boost and MPICH are absent; the
 * rules forbid stand-in headers).  This restatement is pinned by
 *   - the known-answer values the survey measured on the compiled reference
 *     (SURVEY.md §8(a) golden table): weights, h(origin),
 *     first-expansion neighbour sums, z-order owner KAT, final scores,
 *     `-t 1` expansion counts and alignment md5s -> tests/golden/ fixtures;
 *   - the reference's own Cost.cpp + PairAlign.cpp, which compile without
 *     Boost: oracle/Makefile builds them into oracle/_ref/ref_pairalign and
 *     tests/test_oracle.py diffs every PairAlign table against this file.
 */
#include "pastar_oracle.h"

#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

/* ------------------------------------------------------------------ */
/* Cost model                                                          */
/* ------------------------------------------------------------------ */

/* Gap constants, Cost.h:13 (GapExtension = GapOpen = GapGap = 30). */
enum { GAP_EXT = 30, GAP_OPEN = 30, GAP_GAP = 30 };

/* Distance table of Cost.cpp:12-262, lower triangle over the residues
 * "-ACDEFGHIKLMNPQRSTVWY" (the table is symmetric; every other entry of the
 * reference's int[90][90] is zero, Cost.cpp:10).  Note the reference's
 * quirks are data here: C/S/T vs '-' are 0 and W-W is 0.  The same numbers
 * are extracted mechanically into tests/golden/cost_table.json by
 * tools/gen_cost_table.py and cross-checked in tests/test_oracle.py. */
static const char kRes[] = "-ACDEFGHIKLMNPQRSTVWY";
static const signed char kTri[] = {
    0,
    12, 15,
    0, 19, 5,
    12, 17, 22, 13,
    12, 17, 22, 14, 13,
    12, 21, 21, 23, 22, 8,
    12, 16, 20, 16, 17, 22, 12,
    12, 18, 20, 16, 16, 19, 19, 11,
    12, 18, 19, 19, 19, 16, 20, 19, 12,
    12, 18, 22, 17, 17, 22, 19, 17, 19, 12,
    12, 19, 23, 21, 20, 15, 21, 19, 15, 20, 11,
    12, 18, 22, 20, 19, 17, 20, 19, 15, 17, 13, 11,
    12, 17, 21, 15, 16, 21, 17, 15, 19, 16, 20, 19, 15,
    12, 16, 20, 18, 18, 22, 18, 17, 19, 18, 20, 19, 18, 11,
    12, 17, 22, 15, 15, 22, 18, 14, 19, 16, 19, 18, 16, 17, 13,
    12, 19, 21, 18, 18, 21, 20, 15, 19, 14, 20, 17, 17, 17, 16, 11,
    0, 16, 17, 17, 17, 20, 16, 18, 18, 17, 20, 19, 16, 16, 18, 17, 15,
    0, 16, 19, 17, 17, 20, 17, 18, 17, 17, 19, 18, 17, 17, 18, 18, 16, 14,
    12, 17, 19, 19, 19, 18, 18, 19, 13, 19, 15, 15, 19, 18, 19, 19, 18, 17, 13,
    12, 23, 25, 24, 24, 17, 24, 20, 22, 20, 19, 21, 21, 23, 22, 15, 19, 22, 23, 0,
    12, 20, 17, 21, 21, 10, 22, 17, 18, 21, 18, 19, 19, 22, 21, 21, 20, 20, 19, 17, 7,
};

static int g_table[90][90];
static int g_table_ready;

static void build_table(void)
{
    if (g_table_ready)
        return;
    int k = 0;
    for (int i = 0; kRes[i]; i++)
        for (int j = 0; j <= i; j++, k++) {
            int a = (unsigned char)kRes[i], b = (unsigned char)kRes[j];
            g_table[a][b] = g_table[b][a] = kTri[k];
        }
    g_table_ready = 1;
}

/* Cost::cost, Cost.cpp:266-270: pam250[(int)r][(int)l] on an int[90][90].
 * An index >= 90 (e.g. 'Z', lowercase) reads out of bounds in the reference
 * (undefined behaviour); for l >= 90 with r < 89 the flat overflow lands in a
 * column < 45 of the next row, which is always 0, so 0 is the defined value
 * we adopt for every out-of-range residue. */
int orc_cost(int r, int l)
{
    build_table();
    if (r < 0 || l < 0 || r >= 90 || l >= 90)
        return 0;
    return g_table[r][l];
}

static int cost_c(char r, char l) { return orc_cost((int)r, (int)l); }

/* ------------------------------------------------------------------ */
/* Input                                                               */
/* ------------------------------------------------------------------ */

static void add_seq(orc_problem *p, const char *s, int len)
{
    if (p->n >= ORC_MAX_SEQ) {
        p->n++; /* reported as an error by the caller */
        return;
    }
    p->seq[p->n] = (char *)malloc((size_t)len + 1);
    memcpy(p->seq[p->n], s, (size_t)len);
    p->seq[p->n][len] = '\0';
    p->len[p->n] = len;
    p->n++;
}

/* read_fasta_file_core, read_fasta.cpp:8-36: a line that is empty or starts
 * with '>' ends the current sequence; every other line is appended verbatim
 * (a trailing '\r' is kept); empty sequences are dropped. */
orc_problem *orc_load_fasta(const char *path)
{
    FILE *f = fopen(path, "rb");
    if (!f)
        return NULL;
    orc_problem *p = (orc_problem *)calloc(1, sizeof(orc_problem));
    orc_set_gaps(p, GAP_OPEN, GAP_EXT, GAP_GAP);
    size_t cap = 1 << 16, n = 0;
    char *cur = (char *)malloc(cap);
    char *line = NULL;
    size_t lcap = 0;
    ssize_t got;
    while ((got = getline(&line, &lcap, f)) >= 0) {
        size_t ll = (size_t)got;
        if (ll && line[ll - 1] == '\n')
            ll--; /* std::getline strips only '\n' */
        if (ll == 0 || line[0] == '>') {
            if (n)
                add_seq(p, cur, (int)n);
            n = 0;
            continue;
        }
        while (n + ll + 1 > cap) {
            cap *= 2;
            cur = (char *)realloc(cur, cap);
        }
        memcpy(cur + n, line, ll);
        n += ll;
    }
    if (n)
        add_seq(p, cur, (int)n);
    free(cur);
    free(line);
    fclose(f);
    if (p->n < 2 || p->n > ORC_MAX_SEQ) {
        orc_free(p);
        return NULL;
    }
    return p;
}

orc_problem *orc_from_seqs(int n, const char *const *seqs)
{
    if (n < 2 || n > ORC_MAX_SEQ)
        return NULL;
    orc_problem *p = (orc_problem *)calloc(1, sizeof(orc_problem));
    orc_set_gaps(p, GAP_OPEN, GAP_EXT, GAP_GAP);
    for (int i = 0; i < n; i++)
        add_seq(p, seqs[i], (int)strlen(seqs[i]));
    return p;
}

void orc_set_gaps(orc_problem *p, int gap_open, int gap_ext, int gap_gap)
{
    p->gap_open = gap_open;
    p->gap_ext = gap_ext;
    p->gap_gap = gap_gap;
}

void orc_free(orc_problem *p)
{
    if (!p)
        return;
    for (int i = 0; i < p->n && i < ORC_MAX_SEQ; i++)
        free(p->seq[i]);
    for (int k = 0; k < p->npairs; k++)
        free(p->H[k]);
    free(p);
}

/* ------------------------------------------------------------------ */
/* PairAlign (PairAlign.cpp:107-171)                                   */
/* ------------------------------------------------------------------ */

enum { NO_GAP = 0, GAP_X = 1, GAP_Y = 2 };

/* PairAlign::Align + pairCost + gapCost (PairAlign.cpp:85-171).  Fills the
 * suffix table from (l1, l2) back to (0, 0); the affine direction matrix is
 * kept so that patched gap constants keep the reference's tie rules. */
void orc_pairalign(const char *s1, int l1, const char *s2, int l2,
                   int gap_open, int gap_ext, int *M)
{
    const int W = l2 + 1;
    unsigned char *A = (unsigned char *)malloc((size_t)(l1 + 1) * W);
#define MM(i, j) M[(size_t)(i) * W + (j)]
#define AA(i, j) A[(size_t)(i) * W + (j)]
    MM(l1, l2) = 0;
    MM(l1, l2 - 1) = gap_open;
    MM(l1 - 1, l2) = gap_open;
    AA(l1, l2) = NO_GAP;
    AA(l1, l2 - 1) = GAP_Y;
    AA(l1 - 1, l2) = GAP_X;
    for (int j = l2 - 2; j >= 0; j--) {
        MM(l1, j) = MM(l1, j + 1) + gap_ext;
        AA(l1, j) = GAP_Y;
    }
    for (int i = l1 - 2; i >= 0; i--) {
        MM(i, l2) = MM(i + 1, l2) + gap_ext;
        AA(i, l2) = GAP_X;
    }
    for (int i = l1 - 1; i >= 0; i--) {
        for (int j = l2 - 1; j >= 0; j--) {
            int c0 = MM(i + 1, j) + (AA(i + 1, j) == GAP_X ? gap_ext : gap_open);
            int c1 = MM(i, j + 1) + (AA(i, j + 1) == GAP_Y ? gap_ext : gap_open);
            int mn, gv;
            if (c0 < c1) {
                mn = c0;
                gv = GAP_X;
            } else {
                mn = c1;
                gv = GAP_Y;
            }
            int c2 = MM(i + 1, j + 1) + cost_c(s1[i], s2[j]);
            if (c2 < mn) {
                mn = c2;
                gv = NO_GAP;
            }
            MM(i, j) = mn;
            AA(i, j) = (unsigned char)gv;
        }
    }
#undef MM
#undef AA
    free(A);
}

/* ------------------------------------------------------------------ */
/* WeightedSP: Altschul rationale-2 weights (WeightedSP.cpp:109-519)   */
/* ------------------------------------------------------------------ */

#define WSP_BIG 999999
#define WSP_GAP 8
#define WSP_EFGAP 0
enum { DIR_DIAG = 0, DIR_VERT = 1, DIR_HORZ = 2 };
#define INTERNAL_NODE (-1)
#define TREE_ROOT (-2)

static int min3(int a, int b, int c) /* minOf3, WeightedSP.cpp:22-35 */
{
    if (a < b)
        return a < c ? a : c;
    return b < c ? b : c;
}

/* convert_path_to_cost, WeightedSP.cpp:109-142 */
static int path_to_cost(const char *A, const char *B, int n, int m,
                        int **dd, int **hh, int **vv)
{
    int i, j, dir = DIR_DIAG, match = 0;
    for (i = n, j = m; (i || j);) {
        int V = vv[i][j] - (dir == DIR_VERT ? (j == m ? WSP_EFGAP : WSP_GAP) : 0);
        int H = hh[i][j] - (dir == DIR_HORZ ? (i == n ? WSP_EFGAP : WSP_GAP) : 0);
        int M = min3(V, H, dd[i][j]);
        if (!j || M == V) {
            dir = DIR_VERT;
            --i;
        } else if (!i || M == H) {
            dir = DIR_HORZ;
            --j;
        } else {
            dir = DIR_DIAG;
            match += A[i] == B[j];
            --i;
            --j;
        }
    }
    return (int)(0.5 + 1000.0 * (n - match + m - match) / (n + m));
}

/* primer, WeightedSP.cpp:144-244: pairwise end-gap-free distances on the
 * '-'-prefixed sequences.  Returns dist[I][J] (float, symmetric). */
static void primer(int ns, char **S, const int *SL, float *dist)
{
    int maxl = 0;
    for (int k = 0; k < ns; k++)
        if (SL[k] + 1 > maxl)
            maxl = SL[k] + 1;
    int **dd = (int **)malloc(sizeof(int *) * (size_t)maxl);
    int **hh = (int **)malloc(sizeof(int *) * (size_t)maxl);
    int **vv = (int **)malloc(sizeof(int *) * (size_t)maxl);
    for (int k = 0; k < maxl; k++) {
        dd[k] = (int *)calloc((size_t)maxl, sizeof(int));
        hh[k] = (int *)calloc((size_t)maxl, sizeof(int));
        vv[k] = (int *)calloc((size_t)maxl, sizeof(int));
    }
    for (int I = 0; I < ns - 1; I++) {
        const char *A = S[I];
        int n = SL[I];
        for (int J = I + 1; J < ns; J++) {
            const char *B = S[J];
            int m = SL[J];
            dd[0][0] = 0;
            hh[0][0] = vv[0][0] = WSP_EFGAP;
            /* index m / n reads the string terminator: cost(x, '\0') == 0.
             * Row/column m and n are written by the reference but never read
             * back; only indices < n, < m are kept here. */
            for (int j = 1; j < m; j++) {
                vv[0][j] = dd[0][j] = WSP_BIG;
                hh[0][j] = hh[0][j - 1] + cost_c('-', B[j]);
            }
            for (int i = 1; i < n; i++) {
                hh[i][0] = dd[i][0] = WSP_BIG;
                vv[i][0] = vv[i - 1][0] + cost_c(A[i], '-');
            }
            for (int i = 1; i < n; i++) {
                int Gi = (i == (n - 1) ? WSP_EFGAP : WSP_GAP);
                for (int j = 1; j < m; j++) {
                    int Gj = (j == (m - 1) ? WSP_EFGAP : WSP_GAP);
                    dd[i][j] = min3(dd[i - 1][j - 1], hh[i - 1][j - 1], vv[i - 1][j - 1]) +
                               cost_c(A[i], B[j]);
                    hh[i][j] = min3(dd[i][j - 1] + Gi, hh[i][j - 1], vv[i][j - 1] + Gi) +
                               cost_c('-', B[j]);
                    vv[i][j] = min3(dd[i - 1][j] + Gj, hh[i - 1][j] + Gj, vv[i - 1][j]) +
                               cost_c(A[i], '-');
                }
            }
            float d = (float)path_to_cost(A, B, n - 1, m - 1, dd, hh, vv);
            if (d <= 0)
                d = 1;
            dist[(size_t)I * ns + J] = dist[(size_t)J * ns + I] = d;
        }
    }
    for (int k = 0; k < maxl; k++) {
        free(dd[k]);
        free(hh[k]);
        free(vv[k]);
    }
    free(dd);
    free(hh);
    free(vv);
}

typedef struct tnode {
    int parent, left, right, brother;
    float weight, w, W, v, V;
    int seq;
} tnode;

typedef struct wctx {
    tnode *nd;
    int nn;
    const float *D;
    int ns;
} wctx;

static int new_node(wctx *c, int left, int right, int seq)
{
    tnode *t = &c->nd[c->nn];
    t->parent = -1;
    t->left = left;
    t->right = right;
    t->brother = -1;
    t->weight = t->w = t->W = t->v = t->V = 0.0f;
    t->seq = seq;
    return c->nn++;
}

/* compute_path_cost_rec, WeightedSP.cpp:249-264 */
static float pc_rec(wctx *c, int A, int B, int *plen)
{
    if (c->nd[A].seq < 0) {
        ++(*plen);
        return pc_rec(c, c->nd[A].left, B, plen) + pc_rec(c, c->nd[A].right, B, plen);
    } else if (c->nd[B].seq < 0) {
        ++(*plen);
        return pc_rec(c, A, c->nd[B].left, plen) + pc_rec(c, A, c->nd[B].right, plen);
    }
    return c->D[(size_t)c->nd[A].seq * c->ns + c->nd[B].seq];
}

/* compute_path_cost / compute_path_cost_n, WeightedSP.cpp:268-285 */
static float pc_nodes(wctx *c, int A, int B)
{
    int plen = 1;
    float cost = pc_rec(c, A, B, &plen);
    return (float)(cost / plen);
}

/* compute_path_cost_to_leafs, WeightedSP.cpp:56-62 */
static float pc_leafs(wctx *c, int A, float total, int *count2)
{
    if (c->nd[A].seq >= 0)
        return total + c->nd[A].weight;
    (*count2)++;
    float w = c->nd[A].weight;
    return pc_leafs(c, c->nd[A].left, w + total, count2) +
           pc_leafs(c, c->nd[A].right, w + total, count2);
}

/* compute_curr_cost, WeightedSP.cpp:64-76.  `ctl(..., &count2) / count2`
 * reads count2 after the call returns (g++ 11 at -O3 on x86-64). */
static float curr_cost(wctx *c, const int *tree, int nrem, int i, int j)
{
    float diz = 0.0f, djz = 0.0f;
    int count2 = 1;
    for (int t = 0; t < nrem; ++t)
        if (t != i && t != j) {
            diz += pc_nodes(c, tree[i], tree[t]);
            djz += pc_nodes(c, tree[j], tree[t]);
        }
    diz = diz / (nrem - 2);
    djz = djz / (nrem - 2);
    float lhs = (pc_nodes(c, tree[i], tree[j]) + diz - djz) / 2;
    float leafs = pc_leafs(c, tree[i], 0.0f, &count2);
    return lhs - leafs / count2;
}

/* compute_S, WeightedSP.cpp:287-309 */
static float compute_S(wctx *c, const int *tree, int i, int j, int num)
{
    float s1 = 0, s2 = 0;
    for (int t = 0; t < num; t++)
        if (t != i && t != j)
            s1 += pc_nodes(c, tree[i], tree[t]) + pc_nodes(c, tree[j], tree[t]);
    s1 = s1 / (2 * (num - 2));
    for (int t = 0; t < num - 1; t++)
        for (int tt = t + 1; tt < num; tt++)
            if (t != i && t != j && tt != i && tt != j)
                s2 += pc_nodes(c, tree[t], tree[tt]);
    s2 = s2 / (num - 2);
    return (s1 + s2 + pc_nodes(c, tree[i], tree[j]) / 2);
}

/* compute_weights_from_tree, WeightedSP.cpp:405-421 */
static void cwft(wctx *c, float product, float sum, int no, int brother,
                 float *wm, int leaf)
{
    tnode *N = &c->nd[no];
    if (N->seq > INTERNAL_NODE) {
        wm[(size_t)c->nd[leaf].seq * c->ns + N->seq] = sum * product;
    } else if (brother < 0) {
        cwft(c, product * c->nd[N->left].W, sum + c->nd[N->right].weight, N->right, -1, wm, leaf);
        cwft(c, product * c->nd[N->right].W, sum + c->nd[N->left].weight, N->left, -1, wm, leaf);
    } else {
        cwft(c, product * N->V, sum + c->nd[brother].weight, brother, -1, wm, leaf);
        if (N->seq != TREE_ROOT)
            cwft(c, product * c->nd[brother].W, sum + N->weight, N->parent, N->brother, wm, leaf);
    }
}

/* weightAltschulsRationale2, WeightedSP.cpp:424-519 (with
 * phylogeneticThreeNeighborJoin :317-401 and join_nodes :78-107). */
void orc_weights(int ns, const char *const *seqs, float *out)
{
    char **S = (char **)malloc(sizeof(char *) * (size_t)ns);
    int *SL = (int *)malloc(sizeof(int) * (size_t)ns);
    for (int i = 0; i < ns; i++) { /* prepend '-' (:447) */
        int l = (int)strlen(seqs[i]);
        S[i] = (char *)malloc((size_t)l + 2);
        S[i][0] = '-';
        memcpy(S[i] + 1, seqs[i], (size_t)l + 1);
        SL[i] = l + 1;
    }
    float *D = (float *)calloc((size_t)ns * ns, sizeof(float));
    primer(ns, S, SL, D);

    wctx c;
    c.nd = (tnode *)calloc((size_t)(2 * ns + 2), sizeof(tnode));
    c.nn = 0;
    c.D = D;
    c.ns = ns;
    int *tree = (int *)malloc(sizeof(int) * (size_t)ns);
    int *list = (int *)malloc(sizeof(int) * (size_t)(2 * ns + 2));
    int nlist = 0;
    for (int i = 0; i < ns; i++) {
        tree[i] = new_node(&c, -1, -1, i);
        list[nlist++] = tree[i];
    }
    int nrem = ns;
    float mn = (float)1.0E20;
    int min_i = 0, min_j = 0;
    while (nrem > 2) {
        for (int i = 0; i < nrem - 1; i++)
            for (int j = i + 1; j < nrem; j++) {
                float tmp = compute_S(&c, tree, i, j, nrem);
                if (tmp < mn) {
                    min_i = i;
                    min_j = j;
                    mn = tmp;
                }
            }
        /* join_nodes (:78-107) */
        int L = tree[min_i];
        c.nd[L].weight = curr_cost(&c, tree, nrem, min_i, min_j);
        int R = tree[min_j];
        c.nd[R].weight = curr_cost(&c, tree, nrem, min_j, min_i);
        int nw = new_node(&c, L, R, INTERNAL_NODE);
        c.nd[L].brother = R;
        c.nd[R].brother = L;
        c.nd[L].parent = c.nd[R].parent = nw;
        list[nlist++] = nw;
        tree[min_i] = nw;
        tree[min_j] = tree[nrem - 1];
        nrem--;
        mn = (float)1.0E20;
    }
    int L = tree[0], R = tree[1];
    int root = new_node(&c, L, R, TREE_ROOT);
    c.nd[L].brother = R;
    c.nd[R].brother = L;
    c.nd[L].parent = c.nd[R].parent = root;
    list[nlist++] = root;
    {
        int count2 = 1;
        float len = pc_nodes(&c, L, R);
        float t = pc_leafs(&c, L, 0.0f, &count2);
        len -= t / count2;
        count2 = 1;
        t = pc_leafs(&c, R, 0.0f, &count2);
        len -= t / count2;
        c.nd[L].weight = len;
    }

    /* partial weights (:463-495) */
    int p = 0;
    for (; c.nd[list[p]].seq > INTERNAL_NODE; ++p) {
        tnode *no = &c.nd[list[p]];
        no->w = 1.0f;
        no->W = no->weight;
    }
    for (; c.nd[list[p]].seq > TREE_ROOT; ++p) {
        tnode *no = &c.nd[list[p]];
        tnode *l = &c.nd[no->left], *r = &c.nd[no->right];
        no->w = l->w * r->W + l->W * r->w;
        no->W = no->weight * no->w + l->W * r->W;
    }
    c.nd[list[p]].V = 1;
    c.nd[list[p]].v = 0;
    do {
        tnode *no = &c.nd[list[--p]];
        tnode *pa = &c.nd[no->parent], *br = &c.nd[no->brother];
        no->v = pa->v * br->W + pa->V * br->w;
        no->V = no->weight * no->v + pa->V * br->W;
    } while (p != 0);

    float *wm = (float *)calloc((size_t)ns * ns, sizeof(float));
    for (; c.nd[list[p]].seq > INTERNAL_NODE; ++p) {
        tnode *no = &c.nd[list[p]];
        cwft(&c, 1.0f, no->weight, no->parent, no->brother, wm, list[p]);
    }

    /* scale so the smallest pair weight is about 8 (:497-509) */
    float sm = 1.0E+30f;
    for (int j = 1; j < ns; ++j)
        for (int i = 0; i < j; ++i)
            if (wm[(size_t)i * ns + j] < sm)
                sm = wm[(size_t)i * ns + j];
    sm = (float)(sm / 7.9);
    for (int i = 0; i < ns * ns; i++)
        out[i] = 0.0f;
    for (int i = 0; i < ns - 1; ++i)
        for (int j = i + 1; j < ns; ++j) {
            float q = wm[(size_t)i * ns + j] / sm;
            out[(size_t)i * ns + j] = out[(size_t)j * ns + i] = (float)((double)q + 0.5);
        }

    free(wm);
    free(list);
    free(tree);
    free(c.nd);
    free(D);
    for (int i = 0; i < ns; i++)
        free(S[i]);
    free(S);
    free(SL);
}

/* HeuristicHPair::init, HeuristicHPair.cpp:47-67 */
int orc_init_heuristic(orc_problem *p)
{
    int n = p->n;
    if (n < 2 || n > ORC_MAX_SEQ)
        return -1;
    for (int i = 0; i < n; i++)
        if (p->len[i] < 1)
            return -1;
    int k = 0;
    for (int i = 0; i < n - 1; i++)
        for (int j = i + 1; j < n; j++, k++) {
            p->pair_x[k] = i;
            p->pair_y[k] = j;
            p->H[k] = (int *)malloc(sizeof(int) * (size_t)(p->len[i] + 1) * (p->len[j] + 1));
            orc_pairalign(p->seq[i], p->len[i], p->seq[j], p->len[j], p->gap_open, p->gap_ext, p->H[k]);
        }
    p->npairs = k;
    float *w = (float *)malloc(sizeof(float) * (size_t)n * n);
    orc_weights(n, (const char *const *)p->seq, w);
    for (int i = 0; i < n; i++)
        for (int j = 0; j < n; j++)
            p->weight_f[i][j] = w[i * n + j];
    free(w);
    for (k = 0; k < p->npairs; k++)
        p->weight[k] = (int)p->weight_f[p->pair_x[k]][p->pair_y[k]];
    return 0;
}

/* HeuristicHPair::calculate_h, HeuristicHPair.cpp:74-86 */
int orc_h(const orc_problem *p, const uint16_t *pos)
{
    int h = 0;
    for (int k = 0; k < p->npairs; k++) {
        int x = p->pair_x[k], y = p->pair_y[k];
        h += p->H[k][(size_t)pos[x] * (p->len[y] + 1) + pos[y]] * p->weight[k];
    }
    return h;
}

/* ------------------------------------------------------------------ */
/* CoordHash (CoordHash.cpp:28-245)                                    */
/* ------------------------------------------------------------------ */

/* z_order_hash<Shift> (:107-134) over the first `dims` coordinates;
 * part_z_order_hash (:139-166) is the dims == 2 case. */
static unsigned zorder(int dims, const uint16_t *c, int size, int shift)
{
    int hash = 0;
    int bit_to_read = shift / dims;
    unsigned bits = (unsigned)(log2((double)size) + (shift % dims) + 1);
    unsigned total = bits >= 31 ? 0x80000000u : (1u << bits);
    /* bits >= 31 would wrap bit_to_write to 0 and loop forever in the
     * reference; no valid size/shift reaches it (size <= 2^16, shift <= 21). */
    for (unsigned bit_to_write = 1; bit_to_write != 0 && bit_to_write <= total;) {
        for (int j = 0; j < dims && bit_to_write != 0 && bit_to_write <= total; ++j) {
            if (bit_to_read < 16 && (c[j] & (1u << bit_to_read)))
                hash = (int)((unsigned)hash | bit_to_write);
            bit_to_write <<= 1;
        }
        ++bit_to_read;
    }
    return (unsigned)((hash >> (shift % dims)) % size);
}

int orc_get_id(int n, const uint16_t *c, int size, int hash_type, int shift)
{
    if (shift < 0 || shift > 21 || size <= 0)
        return -1;
    switch (hash_type) {
    case ORC_HASH_FSUM: { /* sum_hash (:37-42) */
        unsigned s = 0;
        for (int i = 0; i < n; i++)
            s += c[i];
        return (int)((s >> shift) % (unsigned)size);
    }
    case ORC_HASH_PSUM: { /* part_sum_hash (:52-57) */
        unsigned s = (unsigned)(c[0] + c[1]);
        return (int)((s >> shift) % (unsigned)size);
    }
    case ORC_HASH_PZORDER:
        return (int)zorder(2, c, size, shift);
    case ORC_HASH_FZORDER:
        return (int)zorder(n, c, size, shift);
    default:
        return -1;
    }
}

/* ------------------------------------------------------------------ */
/* Node::getNeigh (Node.cpp:130-248)                                   */
/* ------------------------------------------------------------------ */

void orc_initial_node(const orc_problem *p, orc_node *out)
{
    memset(out, 0, sizeof(*out));
    out->parenti = (1 << p->n) - 1; /* Sequences.cpp:75 */
    out->g = 0;
    out->f = orc_h(p, out->pos);
}

/* Node::pairCost, Node.cpp:130-152 */
static int pair_cost(const orc_problem *p, int m, int mm, int s1, int s2, int parenti)
{
    int b1 = (m >> s1) & 1, b2 = (m >> s2) & 1, s;
    if (b1 && b2)
        return mm;
    if (b1)
        s = s2;
    else if (b2)
        s = s1;
    else
        return p->gap_gap;
    if (((parenti >> s) & 1) != ((m >> s) & 1))
        return p->gap_open;
    return p->gap_ext;
}

int orc_get_neigh(const orc_problem *p, const orc_node *in, int vec_size,
                  int hash_type, int shift, orc_node *out, int *owner)
{
    int n = p->n, np = p->npairs, cnt = 0;
    int mm[ORC_MAX_PAIRS];
    for (int k = 0; k < np; k++) { /* pair tuples (:218-231) */
        int x = p->pair_x[k], y = p->pair_y[k];
        mm[k] = cost_c(p->seq[x][in->pos[x]], p->seq[y][in->pos[y]]);
    }
    int last = (1 << n) - 1;
    for (int m = 1; m <= last; m++) {
        orc_node c;
        memset(&c, 0, sizeof(c));
        int ok = 1;
        for (int i = 0; i < n; i++) { /* Coord::neigh + borderCheck */
            c.pos[i] = (uint16_t)(in->pos[i] + ((m >> i) & 1));
            if (c.pos[i] > p->len[i])
                ok = 0;
        }
        if (!ok)
            continue;
        int costs = 0;
        for (int k = 0; k < np; k++)
            costs += pair_cost(p, m, mm[k], p->pair_x[k], p->pair_y[k], in->parenti) * p->weight[k];
        c.g = in->g + costs;
        c.f = c.g + orc_h(p, c.pos);
        c.parenti = m;
        if (owner)
            owner[cnt] = orc_get_id(n, c.pos, vec_size, hash_type, shift);
        out[cnt++] = c;
    }
    return cnt;
}

/* ------------------------------------------------------------------ */
/* Serial PAStar (-t 1) with Boost.MultiIndex tie order                */
/* ------------------------------------------------------------------ */

/* The OpenList's priority index is ordered_non_unique on f: insert links at
 * the upper bound of the equal range, and modify() (always to a smaller f in
 * conditional_enqueue, PriorityList.h:104-113) either stays in place or is
 * relinked at the upper bound -- in both cases the node ends up last among
 * equal f.  A (f, seq) heap with a fresh seq on every insert/modify and lazy
 * deletion of superseded entries reproduces that order exactly. */

typedef struct rec {
    uint16_t pos[ORC_MAX_SEQ];
    int32_t g, f, parenti;
    uint8_t state; /* 0 none, 1 open, 2 closed */
    uint64_t seq;
} rec;

typedef struct hent {
    int64_t f;
    uint64_t seq;
    uint32_t idx;
} hent;

typedef struct astate {
    int n;
    rec *recs;
    size_t nrec, caprec;
    uint32_t *tab; /* idx+1, 0 = empty */
    size_t tcap;
    hent *heap;
    size_t nheap, capheap;
    uint64_t seq;
} astate;

static uint64_t hash_pos(const uint16_t *pos, int n)
{
    uint64_t h = 0x9E3779B97F4A7C15ull;
    for (int i = 0; i < n; i++) {
        h ^= pos[i];
        h *= 0xBF58476D1CE4E5B9ull;
        h ^= h >> 31;
    }
    return h;
}

static void tab_insert_raw(astate *s, uint32_t idx)
{
    size_t mask = s->tcap - 1, i = hash_pos(s->recs[idx].pos, s->n) & mask;
    while (s->tab[i])
        i = (i + 1) & mask;
    s->tab[i] = idx + 1;
}

static int64_t find_rec(astate *s, const uint16_t *pos)
{
    size_t mask = s->tcap - 1, i = hash_pos(pos, s->n) & mask;
    while (s->tab[i]) {
        rec *r = &s->recs[s->tab[i] - 1];
        if (!memcmp(r->pos, pos, sizeof(uint16_t) * (size_t)s->n))
            return (int64_t)(s->tab[i] - 1);
        i = (i + 1) & mask;
    }
    return -1;
}

static uint32_t new_rec(astate *s, const uint16_t *pos)
{
    if (s->nrec == s->caprec) {
        s->caprec *= 2;
        s->recs = (rec *)realloc(s->recs, sizeof(rec) * s->caprec);
    }
    if ((s->nrec + 1) * 2 > s->tcap) {
        free(s->tab);
        s->tcap *= 2;
        s->tab = (uint32_t *)calloc(s->tcap, sizeof(uint32_t));
        for (size_t k = 0; k < s->nrec; k++)
            tab_insert_raw(s, (uint32_t)k);
    }
    uint32_t idx = (uint32_t)s->nrec++;
    memset(&s->recs[idx], 0, sizeof(rec));
    memcpy(s->recs[idx].pos, pos, sizeof(uint16_t) * (size_t)s->n);
    tab_insert_raw(s, idx);
    return idx;
}

static int hless(const hent *a, const hent *b)
{
    return a->f < b->f || (a->f == b->f && a->seq < b->seq);
}

static void heap_push(astate *s, int64_t f, uint64_t seq, uint32_t idx)
{
    if (s->nheap == s->capheap) {
        s->capheap *= 2;
        s->heap = (hent *)realloc(s->heap, sizeof(hent) * s->capheap);
    }
    size_t i = s->nheap++;
    hent e = {f, seq, idx};
    while (i) {
        size_t pa = (i - 1) / 2;
        if (!hless(&e, &s->heap[pa]))
            break;
        s->heap[i] = s->heap[pa];
        i = pa;
    }
    s->heap[i] = e;
}

static hent heap_pop(astate *s)
{
    hent top = s->heap[0], e = s->heap[--s->nheap];
    size_t i = 0, n = s->nheap;
    for (;;) {
        size_t l = 2 * i + 1, r = l + 1, b = i;
        const hent *best = &e;
        if (l < n && hless(&s->heap[l], best)) {
            b = l;
            best = &s->heap[l];
        }
        if (r < n && hless(&s->heap[r], best))
            b = r;
        if (b == i)
            break;
        s->heap[i] = s->heap[b];
        i = b;
    }
    if (n)
        s->heap[i] = e;
    return top;
}

/* pop the valid minimum; returns -1 if the open list is empty */
static int64_t open_dequeue(astate *s)
{
    while (s->nheap) {
        hent e = heap_pop(s);
        rec *r = &s->recs[e.idx];
        if (r->state == 1 && r->seq == e.seq)
            return (int64_t)e.idx;
    }
    return -1;
}

static int64_t open_min_f(astate *s)
{
    while (s->nheap) {
        hent *e = &s->heap[0];
        rec *r = &s->recs[e->idx];
        if (r->state == 1 && r->seq == e->seq)
            return e->f;
        heap_pop(s);
    }
    return INT64_MAX;
}

/* PAStar::enqueue (PAStar.cpp:219-237) + conditional_enqueue
 * (PriorityList.h:104-113) for one node. */
static void enqueue_node(astate *s, const orc_node *nd, int64_t *reopen)
{
    int64_t fi = find_rec(s, nd->pos);
    uint32_t idx;
    if (fi >= 0) {
        rec *r = &s->recs[fi];
        idx = (uint32_t)fi;
        if (r->state == 2) {
            if (nd->g >= r->g)
                return;
            r->state = 0; /* ClosedList.erase, reopen++ */
            (*reopen)++;
        } else if (r->state == 1) {
            if (nd->f >= r->f)
                return;
            r->f = nd->f; /* modify: f, g, parenti (change_node, Node.h:73-88) */
            r->g = nd->g;
            r->parenti = nd->parenti;
            r->seq = ++s->seq;
            heap_push(s, r->f, r->seq, idx);
            return;
        }
    } else {
        idx = new_rec(s, nd->pos);
    }
    rec *r = &s->recs[idx];
    r->g = nd->g;
    r->f = nd->f;
    r->parenti = nd->parenti;
    r->state = 1;
    r->seq = ++s->seq;
    heap_push(s, r->f, r->seq, idx);
}

static double now_s(void)
{
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return (double)ts.tv_sec + 1e-9 * (double)ts.tv_nsec;
}

int orc_astar(const orc_problem *p, orc_result *res, char *aln, int aln_cap)
{
    int n = p->n;
    memset(res, 0, sizeof(*res));
    astate s;
    memset(&s, 0, sizeof(s));
    s.n = n;
    s.caprec = 1 << 16;
    s.recs = (rec *)malloc(sizeof(rec) * s.caprec);
    s.tcap = 1 << 17;
    s.tab = (uint32_t *)calloc(s.tcap, sizeof(uint32_t));
    s.capheap = 1 << 16;
    s.heap = (hent *)malloc(sizeof(hent) * s.capheap);

    orc_node zero;
    orc_initial_node(p, &zero);
    enqueue_node(&s, &zero, &res->reopen); /* PAStar.cpp:153 */

    uint16_t goal[ORC_MAX_SEQ] = {0};
    for (int i = 0; i < n; i++)
        goal[i] = (uint16_t)p->len[i];
    int masks = 1 << n;
    orc_node *neigh = (orc_node *)malloc(sizeof(orc_node) * (size_t)masks);
    double t0 = now_s();
    int64_t goal_idx = -1;
    int rc = -1;
    for (;;) {
        /* worker_inner, PAStar.cpp:320-401, at one thread */
        int64_t ci = open_dequeue(&s);
        if (ci < 0)
            break;
        res->expansions++; /* nodes_count (:341) counts every dequeue */
        rec *cur = &s.recs[ci];
        cur->state = 2; /* ClosedList[current.pos] = current (:351) */
        if (!memcmp(cur->pos, goal, sizeof(uint16_t) * (size_t)n)) {
            /* process_final_node + check_stop (:410-547) at one rank/thread:
             * accept unless some open node has a strictly smaller f. */
            if (open_min_f(&s) < cur->f) {
                cur->state = 0;
                orc_node g;
                memcpy(g.pos, cur->pos, sizeof(g.pos));
                g.g = cur->g;
                g.f = cur->f;
                g.parenti = cur->parenti;
                enqueue_node(&s, &g, &res->reopen);
                continue;
            }
            goal_idx = ci;
            rc = 0;
            break;
        }
        orc_node node;
        memcpy(node.pos, cur->pos, sizeof(node.pos));
        node.g = cur->g;
        node.f = cur->f;
        node.parenti = cur->parenti;
        int cnt = orc_get_neigh(p, &node, 1, ORC_HASH_FZORDER, 12, neigh, NULL);
        for (int k = 0; k < cnt; k++)
            enqueue_node(&s, &neigh[k], &res->reopen);
    }
    res->seconds = now_s() - t0;
    if (rc == 0) {
        res->score = s.recs[goal_idx].g;
        for (size_t k = 0; k < s.nrec; k++) {
            if (s.recs[k].state == 1)
                res->open_size++;
            else if (s.recs[k].state == 2)
                res->closed_size++;
        }
        /* backtrace_create_alignment (backtrace.cpp:47-69) */
        int cols = 0;
        int64_t idx = goal_idx;
        int cap = 1;
        for (int i = 0; i < n; i++)
            cap += p->len[i];
        char *rows = (char *)malloc((size_t)n * cap);
        uint16_t zero_pos[ORC_MAX_SEQ] = {0};
        while (memcmp(s.recs[idx].pos, zero_pos, sizeof(uint16_t) * (size_t)n)) {
            rec *r = &s.recs[idx];
            uint16_t par[ORC_MAX_SEQ] = {0};
            for (int i = 0; i < n; i++) {
                int moved = (r->parenti >> i) & 1;
                par[i] = (uint16_t)(r->pos[i] - moved);
                rows[(size_t)i * cap + cols] = moved ? p->seq[i][r->pos[i] - 1] : '-';
            }
            cols++;
            idx = find_rec(&s, par);
            if (idx < 0) {
                rc = -2;
                break;
            }
        }
        res->aln_len = cols;
        /* backtrace_print_similarity (backtrace.cpp:136-165) */
        int total = 0, equal = 0;
        for (int col = 0; col < cols; col++)
            for (int i = 0; i < n; i++)
                for (int j = i + 1; j < n; j++) {
                    if (rows[(size_t)i * cap + col] == rows[(size_t)j * cap + col])
                        ++equal;
                    ++total;
                }
        res->similarity = total ? (double)((float)(equal * 100) / (float)total) : 0.0;
        if (aln && aln_cap > cols) {
            for (int i = 0; i < n; i++) {
                for (int col = 0; col < cols; col++)
                    aln[(size_t)i * aln_cap + col] = rows[(size_t)i * cap + (cols - 1 - col)];
                aln[(size_t)i * aln_cap + cols] = '\0';
            }
        }
        free(rows);
    }
    free(neigh);
    free(s.recs);
    free(s.tab);
    free(s.heap);
    return rc;
}

int64_t orc_alignment_cost(const orc_problem *p, const char *aln, int stride, int cols)
{
    int n = p->n;
    uint16_t pos[ORC_MAX_SEQ] = {0};
    int parenti = (1 << n) - 1;
    int64_t g = 0;
    for (int col = 0; col < cols; col++) {
        int m = 0;
        for (int i = 0; i < n; i++)
            if (aln[(size_t)i * stride + col] != '-')
                m |= 1 << i;
        if (!m)
            return -1;
        for (int k = 0; k < p->npairs; k++) {
            int x = p->pair_x[k], y = p->pair_y[k];
            int mm = cost_c(p->seq[x][pos[x]], p->seq[y][pos[y]]);
            g += (int64_t)pair_cost(p, m, mm, x, y, parenti) * p->weight[k];
        }
        for (int i = 0; i < n; i++)
            pos[i] = (uint16_t)(pos[i] + ((m >> i) & 1));
        parenti = m;
    }
    for (int i = 0; i < n; i++)
        if (pos[i] != p->len[i])
            return -1;
    return g;
}

/* ------------------------------------------------------------------ */
/* Multithreaded PAStar (the reference's -t T, one rank)               */
/* ------------------------------------------------------------------ */

/* PAStar<N>::worker_inner (PAStar.cpp:320-401) over T threads: thread t owns
 * the coordinates with get_id(c, T) == t (FZORDER, shift 12, Node.cpp:244);
 * each holds its own open and closed lists (an astate, as in orc_astar) and
 * an inbox that the other threads append to (the reference's per-thread
 * queue_mutex-protected vectors, PAStar.cpp:366-396).  Used as the timed
 * multicore CPU baseline (-t $(nproc)); expansions and
 * order are non-deterministic, the score is exact.
 *
 * Goal and stop (PAStar.cpp:410-547, restated): the goal's owner records
 * g(goal) in `best` when it pops it (h(goal) = 0); a node with f >= best is
 * never expanded.  A thread is idle when its open list has nothing below
 * best and its inbox and outgoing buffers are empty.  Termination is the
 * counting test: read the received count, then every idle flag, then the
 * sent count; stop iff all idle and received == sent.  Senders count a
 * message before it becomes visible, and a receiver clears its idle flag
 * before it counts a receipt, which makes the test sound. */

#include <pthread.h>
#include <sched.h>
#include <stdatomic.h>

typedef struct mt_inbox {
    pthread_mutex_t mu;
    orc_node *v;
    size_t n, cap;
    atomic_llong avail; /* n, readable without the lock (a hint) */
} mt_inbox;

typedef struct mt_shared {
    const orc_problem *p;
    int T;
    mt_inbox *inbox;
    atomic_int *idle;
    atomic_llong sent, received, best, expansions, reopen;
    atomic_int stop;
} mt_shared;

typedef struct mt_arg {
    mt_shared *sh;
    int t;
} mt_arg;

static void vec_push(orc_node **v, size_t *n, size_t *cap, const orc_node *x)
{
    if (*n == *cap) {
        *cap = *cap ? *cap * 2 : 256;
        *v = (orc_node *)realloc(*v, sizeof(orc_node) * *cap);
    }
    (*v)[(*n)++] = *x;
}

static void mt_flush(mt_shared *sh, orc_node **out, size_t *out_n, size_t *out_cap)
{
    for (int d = 0; d < sh->T; d++) {
        if (!out_n[d])
            continue;
        atomic_fetch_add(&sh->sent, (long long)out_n[d]); /* counted before visible */
        mt_inbox *ib = &sh->inbox[d];
        pthread_mutex_lock(&ib->mu);
        for (size_t k = 0; k < out_n[d]; k++)
            vec_push(&ib->v, &ib->n, &ib->cap, &out[d][k]);
        atomic_store(&ib->avail, (long long)ib->n);
        pthread_mutex_unlock(&ib->mu);
        out_n[d] = 0;
    }
    (void)out_cap;
}

static void *mt_worker(void *argp)
{
    mt_arg *arg = (mt_arg *)argp;
    mt_shared *sh = arg->sh;
    const orc_problem *p = sh->p;
    const int t = arg->t, T = sh->T, n = p->n;
    astate s;
    memset(&s, 0, sizeof(s));
    s.n = n;
    s.caprec = 1 << 14;
    s.recs = (rec *)malloc(sizeof(rec) * s.caprec);
    s.tcap = 1 << 15;
    s.tab = (uint32_t *)calloc(s.tcap, sizeof(uint32_t));
    s.capheap = 1 << 14;
    s.heap = (hent *)malloc(sizeof(hent) * s.capheap);
    orc_node **out = (orc_node **)calloc((size_t)T, sizeof(orc_node *));
    size_t *out_n = (size_t *)calloc((size_t)T, sizeof(size_t));
    size_t *out_cap = (size_t *)calloc((size_t)T, sizeof(size_t));
    orc_node *drain = NULL;
    size_t drain_cap = 0;
    orc_node *neigh = (orc_node *)malloc(sizeof(orc_node) * ((size_t)1 << n));
    int *owner = (int *)malloc(sizeof(int) * ((size_t)1 << n));
    uint16_t goal[ORC_MAX_SEQ] = {0};
    for (int i = 0; i < n; i++)
        goal[i] = (uint16_t)p->len[i];
    int64_t expansions = 0, reopen = 0;
    int since_flush = 0;
    while (!atomic_load(&sh->stop)) {
        /* consume the inbox (PAStar::enqueue of received nodes) */
        mt_inbox *ib = &sh->inbox[t];
        size_t got = 0;
        if (atomic_load(&ib->avail)) {
            pthread_mutex_lock(&ib->mu);
            got = ib->n;
            if (got) {
                orc_node *tmp = ib->v;
                size_t tcap = ib->cap;
                ib->v = drain;
                ib->cap = drain_cap;
                ib->n = 0;
                drain = tmp;
                drain_cap = tcap;
            }
            atomic_store(&ib->avail, 0);
            pthread_mutex_unlock(&ib->mu);
        }
        if (got) {
            atomic_store(&sh->idle[t], 0); /* before the receipt is counted */
            atomic_fetch_add(&sh->received, (long long)got);
            long long best = atomic_load(&sh->best);
            for (size_t k = 0; k < got; k++)
                if (drain[k].f < best)
                    enqueue_node(&s, &drain[k], &reopen);
        }
        long long best = atomic_load(&sh->best);
        if (open_min_f(&s) < best) {
            atomic_store(&sh->idle[t], 0);
            int64_t ci = open_dequeue(&s);
            expansions++;
            rec *cur = &s.recs[ci];
            cur->state = 2;
            if (!memcmp(cur->pos, goal, sizeof(uint16_t) * (size_t)n)) {
                long long g = cur->g, old = atomic_load(&sh->best);
                while (g < old && !atomic_compare_exchange_weak(&sh->best, &old, g))
                    ;
                continue;
            }
            orc_node node;
            memcpy(node.pos, cur->pos, sizeof(node.pos));
            node.g = cur->g;
            node.f = cur->f;
            node.parenti = cur->parenti;
            int cnt = orc_get_neigh(p, &node, T, ORC_HASH_FZORDER, 12, neigh, owner);
            for (int k = 0; k < cnt; k++) {
                if (neigh[k].f >= best)
                    continue;
                if (owner[k] == t)
                    enqueue_node(&s, &neigh[k], &reopen);
                else
                    vec_push(&out[owner[k]], &out_n[owner[k]], &out_cap[owner[k]], &neigh[k]);
            }
            if (++since_flush >= 8) {
                mt_flush(sh, out, out_n, out_cap);
                since_flush = 0;
            }
            continue;
        }
        /* nothing below best here: hand over what is buffered, go idle */
        mt_flush(sh, out, out_n, out_cap);
        since_flush = 0;
        pthread_mutex_lock(&ib->mu);
        int empty = ib->n == 0;
        if (empty)
            atomic_store(&sh->idle[t], 1);
        pthread_mutex_unlock(&ib->mu);
        if (!empty)
            continue;
        /* counting termination test */
        long long r = atomic_load(&sh->received);
        int all = 1;
        for (int d = 0; d < T && all; d++)
            all = atomic_load(&sh->idle[d]);
        long long sn = atomic_load(&sh->sent);
        if (all && r == sn) {
            atomic_store(&sh->stop, 1);
            break;
        }
        sched_yield();
    }
    atomic_fetch_add(&sh->expansions, expansions);
    atomic_fetch_add(&sh->reopen, reopen);
    for (int d = 0; d < T; d++)
        free(out[d]);
    free(out);
    free(out_n);
    free(out_cap);
    free(drain);
    free(neigh);
    free(owner);
    free(s.recs);
    free(s.tab);
    free(s.heap);
    return NULL;
}

int orc_pastar_mt(const orc_problem *p, int threads, orc_result *res)
{
    memset(res, 0, sizeof(*res));
    if (threads < 1 || threads > 1024)
        return -1;
    mt_shared sh;
    memset(&sh, 0, sizeof(sh));
    sh.p = p;
    sh.T = threads;
    sh.inbox = (mt_inbox *)calloc((size_t)threads, sizeof(mt_inbox));
    sh.idle = (atomic_int *)calloc((size_t)threads, sizeof(atomic_int));
    for (int t = 0; t < threads; t++)
        pthread_mutex_init(&sh.inbox[t].mu, NULL);
    atomic_store(&sh.best, INT64_MAX);
    /* the origin on its owner (PAStar.cpp:153) */
    orc_node zero;
    orc_initial_node(p, &zero);
    int own0 = orc_get_id(p->n, zero.pos, threads, ORC_HASH_FZORDER, 12);
    atomic_fetch_add(&sh.sent, 1);
    vec_push(&sh.inbox[own0].v, &sh.inbox[own0].n, &sh.inbox[own0].cap, &zero);
    atomic_store(&sh.inbox[own0].avail, 1);
    pthread_t *th = (pthread_t *)malloc(sizeof(pthread_t) * (size_t)threads);
    mt_arg *args = (mt_arg *)malloc(sizeof(mt_arg) * (size_t)threads);
    double t0 = now_s();
    for (int t = 0; t < threads; t++) {
        args[t].sh = &sh;
        args[t].t = t;
        pthread_create(&th[t], NULL, mt_worker, &args[t]);
    }
    for (int t = 0; t < threads; t++)
        pthread_join(th[t], NULL);
    res->seconds = now_s() - t0;
    res->expansions = atomic_load(&sh.expansions);
    res->reopen = atomic_load(&sh.reopen);
    long long best = atomic_load(&sh.best);
    res->score = best;
    for (int t = 0; t < threads; t++) {
        free(sh.inbox[t].v);
        pthread_mutex_destroy(&sh.inbox[t].mu);
    }
    free(sh.inbox);
    free((void *)sh.idle);
    free(th);
    free(args);
    return best == INT64_MAX ? -1 : 0;
}
