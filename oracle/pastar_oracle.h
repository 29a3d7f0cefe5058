/*
 * pastar_oracle.h -- CPU restatement of the reference PAStar hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  This is the parity oracle: only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it, and
 * only as the checker (or the timed CPU baseline), never as the product path.
 * The product (mpi_pastar_msa_amd/csrc) never links or calls anything here.
 *
 * Every function restates a reference function; the file:line it follows is
 * cited at each definition in pastar_oracle.c.  Parity pinning: see the header
 * of pastar_oracle.c.
 */
#ifndef PASTAR_ORACLE_H
#define PASTAR_ORACLE_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define ORC_MAX_SEQ 16
#define ORC_MAX_PAIRS (ORC_MAX_SEQ * (ORC_MAX_SEQ - 1) / 2)

enum { ORC_HASH_FZORDER = 0, ORC_HASH_PZORDER = 1, ORC_HASH_FSUM = 2, ORC_HASH_PSUM = 3 };

typedef struct orc_problem {
    int n;                          /* number of sequences (3..16)          */
    int len[ORC_MAX_SEQ];           /* residues per sequence                */
    char *seq[ORC_MAX_SEQ];         /* NUL-terminated residue strings       */
    float weight_f[ORC_MAX_SEQ][ORC_MAX_SEQ]; /* Altschul rationale-2 weights */
    int weight[ORC_MAX_PAIRS];      /* (int)weight_f[x][y], pair order      */
    int pair_x[ORC_MAX_PAIRS], pair_y[ORC_MAX_PAIRS];
    int npairs;
    int *H[ORC_MAX_PAIRS];          /* PairAlign suffix tables, row-major   */
    int gap_open, gap_ext, gap_gap; /* Cost.h:13 (all 30); patchable so the
                                       general pairCost form can be checked */
} orc_problem;

typedef struct orc_node {
    uint16_t pos[ORC_MAX_SEQ];
    int32_t g, f, parenti;
} orc_node;

typedef struct orc_result {
    int64_t score;          /* g of the goal                          */
    int64_t expansions;     /* dequeues incl. the goal (PAStar Total) */
    int64_t reopen;
    int64_t open_size, closed_size;
    double similarity;      /* percent, as printed by the reference   */
    double seconds;         /* first dequeue -> goal accepted         */
    int aln_len;            /* alignment columns                      */
} orc_result;

/* Cost::cost (Cost.cpp:266-270) */
int orc_cost(int r, int l);

/* FASTA reader + Sequences (read_fasta.cpp:8-36, Sequences.cpp:53-65).
 * Returns NULL on error. */
orc_problem *orc_load_fasta(const char *path);
orc_problem *orc_from_seqs(int n, const char *const *seqs);
void orc_free(orc_problem *p);

/* Patch the gap constants (Cost.h:13) before orc_init_heuristic. */
void orc_set_gaps(orc_problem *p, int gap_open, int gap_ext, int gap_gap);

/* Phase 1: HeuristicHPair::init (HeuristicHPair.cpp:47-67). */
int orc_init_heuristic(orc_problem *p);

/* PairAlign::Align, one pair (PairAlign.cpp:137-171); out is (l1+1)*(l2+1). */
void orc_pairalign(const char *s1, int l1, const char *s2, int l2,
                   int gap_open, int gap_ext, int *out);

/* weightAltschulsRationale2 (WeightedSP.cpp:424-519); out is n*n floats. */
void orc_weights(int n, const char *const *seqs, float *out);

/* HeuristicHPair::calculate_h (HeuristicHPair.cpp:74-86) */
int orc_h(const orc_problem *p, const uint16_t *pos);

/* Coord::get_id (CoordHash.cpp:191-245) with the hash configured by
 * Coord::configure_hash.  Returns -1 on an invalid shift (the reference
 * throws std::invalid_argument). */
int orc_get_id(int n, const uint16_t *pos, int size, int hash_type, int shift);

/* Node::getNeigh (Node.cpp:206-248): appends valid neighbours in mask order,
 * writes their owner get_id(vec_size).  Returns the count. */
int orc_get_neigh(const orc_problem *p, const orc_node *in, int vec_size,
                  int hash_type, int shift, orc_node *out, int *owner);

/* Initial node (Sequences.cpp:70-77) */
void orc_initial_node(const orc_problem *p, orc_node *out);

/* Serial PAStar at -t 1 (PAStar.cpp:320-401, PriorityList.h:84-113,
 * AStar.cpp:54-104).  aln receives n rows of aln_cap chars each (may be NULL).
 * Returns 0 on success. */
int orc_astar(const orc_problem *p, orc_result *res, char *aln, int aln_cap);

/* Multithreaded PAStar (-t threads, one rank; PAStar.cpp:320-547): z-order
 * owned open/closed lists per thread, inbox exchange, counting termination.
 * The timed multicore CPU baseline; score exact, expansions vary run to run.
 * Returns 0 on success. */
int orc_pastar_mt(const orc_problem *p, int threads, orc_result *res);

/* SP cost of a given alignment (rows of equal length) under the same
 * weighted edge costs (Node.cpp:130-152 summed along the path). */
int64_t orc_alignment_cost(const orc_problem *p, const char *aln, int aln_stride, int cols);

#ifdef __cplusplus
}
#endif
#endif
