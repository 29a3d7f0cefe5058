// lists_astar_main.cpp -- the reference's serial worker loop (worker_inner,
// PAStar.cpp:320-401, at one thread) written against the OpenList /
// ClosedList facades of include/pastar_lists.hpp: every list operation goes
// through the C-ABI to the device lists, getNeigh to the expand kernel.  It
// shows the drop-in at the list level and is the parity test of that API
// (tests/test_gpu_lists.py).
//
//   pastar_lists_astar <fasta>    prints the reference's "Final Score" line,
//                                 then "expansions <n> reopen <n>"
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "pastar_gpu.h"
#include "pastar_lists.hpp"

namespace {

template <int N>
int run(pastar_ctx *ctx, const std::vector<int> &lengths)
{
    pastar::PriorityList<N> open(ctx);
    pastar::ClosedList<N> closed(ctx);
    const int n = (int)lengths.size();
    // the origin (Sequences::get_initial_node, Sequences.cpp:70-77)
    pastar_node origin{};
    pastar::check(pastar_gpu_h(ctx, origin.pos, 1, &origin.f));
    origin.g = 0;
    origin.parent_mask = (1 << n) - 1;
    open.conditional_enqueue(origin);
    std::vector<pastar_node> neigh((size_t)1 << n);
    long long expansions = 0, reopen = 0;
    for (;;) {
        pastar_node cur;
        if (!open.dequeue(cur)) {
            std::fprintf(stderr, "OpenList exhausted without reaching the final coordinate\n");
            return 1;
        }
        expansions++;  // nodes_count (:341)
        bool final = true;
        for (int i = 0; i < n; i++)
            final &= cur.pos[i] == lengths[i];
        if (final) {
            // process_final_node + check_stop at one thread (:410-547): the
            // goal stands unless the OpenList holds a smaller f
            if (open.get_highest_priority() < cur.f) {
                closed.erase(cur.pos);
                open.conditional_enqueue(cur);
                continue;
            }
            std::printf("Final Score: (");
            for (int i = 0; i < n; i++)
                std::printf(i ? " %d" : "%d", cur.pos[i]);
            std::printf(")\tg - %d (h - 0 f - %d)\n", cur.g, cur.f);
            std::printf("expansions %lld reopen %lld open %zu closed %zu\n", expansions,
                        reopen + (long long)open.reopened(), open.size(), closed.size());
            return 0;
        }
        // Node::getNeigh (Node.cpp:206-248) on the device, then PAStar::enqueue
        int64_t cnt = 0;
        pastar::check(pastar_gpu_expand(ctx, &cur, 1, 1, neigh.data(), nullptr, nullptr, &cnt));
        open.enqueue(std::vector<pastar_node>(neigh.begin(), neigh.begin() + cnt));
    }
}

}  // namespace

int main(int argc, char **argv)
{
    if (argc != 2) {
        std::fprintf(stderr, "usage: %s <fasta>\n", argv[0]);
        return 2;
    }
    int n = PASTAR_MAX_SEQ;
    std::vector<int> lengths(PASTAR_MAX_SEQ);
    std::vector<char> buf(1 << 20);
    if (pastar_read_fasta(argv[1], buf.data(), (int64_t)buf.size(), &n, lengths.data()) != PASTAR_OK) {
        std::fprintf(stderr, "%s\n", pastar_last_error());
        return 1;
    }
    lengths.resize((size_t)n);
    std::vector<const char *> res((size_t)n);
    size_t off = 0;
    for (int i = 0; i < n; i++) {
        res[(size_t)i] = buf.data() + off;
        off += (size_t)lengths[(size_t)i];
    }
    pastar_problem p{};
    p.n = n;
    p.lengths = lengths.data();
    p.residues = res.data();
    p.gap_open = p.gap_ext = p.gap_gap = 30;
    p.hash_type = PASTAR_HASH_FZORDER;
    p.hash_shift = 12;
    pastar_ctx *ctx = nullptr;
    if (pastar_gpu_create(&p, 0, 1, 0, nullptr, &ctx) != PASTAR_OK ||
        pastar_gpu_build_heuristic(ctx) != PASTAR_OK) {
        std::fprintf(stderr, "%s\n", pastar_last_error());
        return 1;
    }
    int rc = 1;
    try {
        switch (n) {
        case 2: rc = run<2>(ctx, lengths); break;
        case 3: rc = run<3>(ctx, lengths); break;
        case 4: rc = run<4>(ctx, lengths); break;
        case 5: rc = run<5>(ctx, lengths); break;
        case 6: rc = run<6>(ctx, lengths); break;
        case 7: rc = run<7>(ctx, lengths); break;
        case 8: rc = run<8>(ctx, lengths); break;
        default: std::fprintf(stderr, "2..8 sequences\n"); break;
        }
    } catch (const pastar::Error &e) {
        std::fprintf(stderr, "%s\n", e.what());
        rc = 1;
    }
    pastar_gpu_destroy(ctx);
    return rc;
}
