/*
 * oracle_main.c -- command-line driver of the CPU oracle (test infrastructure).
 *
 *   pastar_oracle FILE.fasta          reference-style report (msa_pastar -t 1)
 *   pastar_oracle --json FILE.fasta   machine-readable summary for fixtures
 *
 * The reference-style report follows the line order of msa_pastar at one
 * thread (HeuristicHPair.cpp:52-63, Node.cpp:41-47, backtrace.cpp:136-191,
 * PAStar.cpp:591-619); timing lines are omitted.
 */
#include "pastar_oracle.h"

#include <stdio.h>
#include <stdlib.h>
#include <string.h>

int main(int argc, char **argv)
{
    int json = 0;
    const char *path = NULL;
    for (int i = 1; i < argc; i++) {
        if (!strcmp(argv[i], "--json"))
            json = 1;
        else
            path = argv[i];
    }
    if (!path) {
        fprintf(stderr, "usage: %s [--json] file.fasta\n", argv[0]);
        return 2;
    }
    orc_problem *p = orc_load_fasta(path);
    if (!p) {
        fprintf(stderr, "Can't open file %s\n", path);
        return 1;
    }
    if (orc_init_heuristic(p)) {
        fprintf(stderr, "invalid input\n");
        return 1;
    }
    int n = p->n, cap = 1;
    for (int i = 0; i < n; i++)
        cap += p->len[i];
    char *aln = (char *)malloc((size_t)n * cap);
    orc_result r;
    int rc = orc_astar(p, &r, aln, cap);
    if (rc) {
        fprintf(stderr, "search failed (%d)\n", rc);
        return 1;
    }
    orc_node zero, *nb = (orc_node *)malloc(sizeof(orc_node) << n);
    orc_initial_node(p, &zero);
    int cnt = orc_get_neigh(p, &zero, 1, 0, 12, nb, NULL);
    long long sg = 0, sh = 0;
    for (int k = 0; k < cnt; k++) {
        sg += nb[k].g;
        sh += nb[k].f - nb[k].g;
    }
    if (json) {
        printf("{\"n\": %d, \"lengths\": [", n);
        for (int i = 0; i < n; i++)
            printf("%s%d", i ? ", " : "", p->len[i]);
        printf("], \"weights\": [");
        for (int k = 0; k < p->npairs; k++)
            printf("%s%d", k ? ", " : "", p->weight[k]);
        printf("], \"h_origin\": %d, \"first_expansion\": {\"count\": %d, \"sum_g\": %lld, "
               "\"sum_h\": %lld}, \"score\": %lld, \"expansions\": %lld, \"reopen\": %lld, "
               "\"similarity\": \"%.2f\", \"seconds\": %.6f, \"alignment\": [",
               zero.f, cnt, sg, sh, (long long)r.score, (long long)r.expansions,
               (long long)r.reopen, r.similarity, r.seconds);
        for (int i = 0; i < n; i++)
            printf("%s\"%s\"", i ? ", " : "", aln + (size_t)i * cap);
        printf("]}\n");
    } else {
        printf("Starting pairwise alignments... done!\n");
        printf("Performing search with Parallel A-Star.\n");
        printf("Running PAStar with: 1 threads (1 machines with 1 threads each),"
               "Full-Zorder hash, 12 shift.\n");
        printf("Final Score: (");
        for (int i = 0; i < n; i++)
            printf("%s%d", i ? " " : "", p->len[i]);
        printf(")\tg - %lld (h - 0 f - %lld)\n", (long long)r.score, (long long)r.score);
        printf("Similarity: %.2f%%\n", r.similarity);
        printf("\n");
        for (int i = 0; i < n; i++)
            printf("%s\n", aln + (size_t)i * cap);
        printf("Total nodes count:\n");
        printf("tid 0\tOpenList:%lld\tClosedList:%lld\tReopen:%lld\tTotal: %lld\n",
               (long long)r.open_size, (long long)r.closed_size, (long long)r.reopen,
               (long long)r.expansions);
        printf("Sum\tOpenList:%lld\tClosedList:%lld\tReopen:%lld\tTotal: %lld\n",
               (long long)r.open_size, (long long)r.closed_size, (long long)r.reopen,
               (long long)r.expansions);
    }
    free(nb);
    free(aln);
    orc_free(p);
    return 0;
}
