// msa_pastar_main.cpp -- the msa_pastar command line on top of the C-ABI.
//
// Mirrors the reference CLI (msa_pastar_main.cpp:56-193, msa_options.cpp:24-160):
//   msa_pastar [-t THREADS] [-s SHIFT] [-y FZORDER|FSUM|PZORDER|PSUM]
//              [--memory_debug] [-v] [-h] file.fasta
// and its report (HeuristicHPair.cpp:52-63, PAStar.cpp:106-113, Node.cpp:41-47,
// backtrace.cpp:20-191, PAStar.cpp:591-619).  MPI ranks become GPU shards:
//   --gpus G   one process per GPU (forked before any HIP call), nodes routed
//              by the same z-order owner hash, exchanged over RCCL.
// Engine knobs: --batch K, --table-log2 L, --pool E, --verbose.
#include <sys/ioctl.h>
#include <sys/wait.h>
#include <unistd.h>

#include <chrono>
#include <climits>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <iomanip>
#include <iostream>
#include <string>
#include <vector>

#include "pastar_gpu.h"

namespace {

struct Options {
    int threads = 1;
    int hash_shift = 12;
    int hash_type = PASTAR_HASH_FZORDER;
    int gpus = 1;
    long long batch = 0, table_log2 = 0, pool = 0;
    bool verbose = false;
    std::string file;
};

const char *kHashName[] = {"Full-Zorder", "Partial-Zorder", "Full-Sum", "Partial-Sum"};

void usage(const char *argv0)
{
    std::cout << "Usage " << argv0 << " [OPTIONS] file.fasta:\n"
              << "Options:\n"
              << "  -v [ --version ]          print version string\n"
              << "  -h [ --help ]             produce help message\n"
              << "  --memory_debug            memory debug option\n\n"
              << "Parallel Options:\n"
              << "  -t [ --threads ] arg (=1) number of threads\n"
              << "  -s [ --hash_shift ] arg (=12) Hash shift option value\n"
              << "  -y [ --hash_type ] arg (=FZORDER) Hash type [FZORDER|FSUM|PZORDER|PSUM]\n"
              << "  --gpus arg (=1)           GPU shards (one process per GPU)\n"
              << "  --batch arg               open nodes expanded per step\n"
              << "  --table-log2 arg          node table capacity (log2 slots)\n"
              << "  --pool arg                open-list entry pool (entries)\n"
              << std::endl;
}

// msa_options_core (msa_options.cpp:24-120).  Returns 0 ok, 1 usage, -1 error.
int parse(int argc, char **argv, Options &o)
{
    auto need = [&](int &i) -> const char * {
        if (i + 1 >= argc) {
            std::cerr << "Invalid argument: the required argument for option '" << argv[i] << "' is missing\n";
            return nullptr;
        }
        return argv[++i];
    };
    bool help = false;
    for (int i = 1; i < argc; i++) {
        std::string a = argv[i];
        const char *v = nullptr;
        if (a == "-v" || a == "--version") {
            std::cout << "msa_pastar, version 1.0\n";
            std::exit(0);
        } else if (a == "-h" || a == "--help") {
            help = true;
        } else if (a == "--memory_debug" || a == "--verbose") {
            o.verbose |= a == "--verbose";
        } else if (a == "-t" || a == "--threads") {
            if (!(v = need(i)))
                return -1;
            o.threads = std::atoi(v);
        } else if (a == "-s" || a == "--hash_shift") {
            if (!(v = need(i)))
                return -1;
            o.hash_shift = std::atoi(v);
        } else if (a == "-y" || a == "--hash_type") {
            if (!(v = need(i)))
                return -1;
            std::string h = v;
            if (h == "FZORDER")
                o.hash_type = PASTAR_HASH_FZORDER;
            else if (h == "FSUM")
                o.hash_type = PASTAR_HASH_FSUM;
            else if (h == "PZORDER")
                o.hash_type = PASTAR_HASH_PZORDER;
            else if (h == "PSUM")
                o.hash_type = PASTAR_HASH_PSUM;
            else {
                std::cerr << "Invalid argument: the argument ('" << h << "') for option '--hash_type' is invalid\n";
                return -1;
            }
        } else if (a == "--gpus") {
            if (!(v = need(i)))
                return -1;
            o.gpus = std::atoi(v);
        } else if (a == "--batch") {
            if (!(v = need(i)))
                return -1;
            o.batch = std::atoll(v);
        } else if (a == "--table-log2") {
            if (!(v = need(i)))
                return -1;
            o.table_log2 = std::atoll(v);
        } else if (a == "--pool") {
            if (!(v = need(i)))
                return -1;
            o.pool = std::atoll(v);
        } else if (!a.empty() && a[0] == '-') {
            std::cerr << "Invalid argument: unrecognised option '" << a << "'\n";
            return -1;
        } else {
            o.file = a;
        }
    }
    if (help || o.file.empty()) {
        usage(argv[0]);
        return 1;
    }
    if (access(o.file.c_str(), R_OK) != 0) {
        std::cout << "File: " << o.file << " is not a regular file.\n";
        return 1;
    }
    return 0;
}

std::string mmss(double s)  // TimeCounter (TimeCounter.cpp:15-26)
{
    long long ms = (long long)(s * 1000.0);
    char buf[64];
    std::snprintf(buf, sizeof(buf), "%02lld:%02lld.%03lld s", ms / 60000, (ms / 1000) % 60, ms % 1000);
    return buf;
}

double now()
{
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int print_width()  // get_print_size (backtrace.cpp:20-35)
{
    if (!isatty(1))
        return INT_MAX;
    struct winsize w;
    if (ioctl(0, TIOCGWINSZ, &w) == 0 && w.ws_col > 1)
        return w.ws_col - 1;
    return 80;
}

struct ShardReport {
    pastar_result r;
    int status;
};

#define CHECK(expr)                                                                  \
    do {                                                                             \
        int _rc = (expr);                                                            \
        if (_rc != PASTAR_OK) {                                                      \
            std::cerr << "Running fatal error: " << pastar_last_error() << std::endl; \
            return 1;                                                                \
        }                                                                            \
    } while (0)

// One shard's whole run (pa_star_run_core, msa_pastar_main.cpp:20-37).
int run_shard(const Options &o, int rank, const unsigned char *rid, ShardReport *report)
{
    std::vector<char> buf(1 << 22);
    int n = PASTAR_MAX_SEQ;
    int lengths[PASTAR_MAX_SEQ];
    const int rc = pastar_read_fasta(o.file.c_str(), buf.data(), (int64_t)buf.size(), &n, lengths);
    if (rc == PASTAR_EIO) {
        std::cout << "Can't open file " << o.file << std::endl;
        return 1;
    }
    CHECK(rc);
    if (n < 3 || n > PASTAR_MAX_SEQ) {
        std::cerr << "Fatal error: Invalid number of sequences: " << n << std::endl;
        return 1;
    }
    std::vector<std::string> seqs;
    const char *res[PASTAR_MAX_SEQ];
    size_t off = 0;
    for (int i = 0; i < n; i++) {
        seqs.emplace_back(buf.data() + off, (size_t)lengths[i]);
        off += (size_t)lengths[i];
    }
    for (int i = 0; i < n; i++)
        res[i] = seqs[i].data();
    pastar_problem p{};
    p.n = n;
    p.lengths = lengths;
    p.residues = res;
    p.weights = nullptr;
    p.sub = nullptr;
    p.gap_open = p.gap_ext = p.gap_gap = 30;
    p.hash_type = o.hash_type;
    p.hash_shift = o.hash_shift;
    const bool lead = rank == 0;

    pastar_ctx *ctx = nullptr;
    double t = now();
    if (lead)
        std::cout << "Starting pairwise alignments... " << std::flush;
    CHECK(pastar_gpu_create(&p, rank, o.gpus, rank, o.gpus > 1 ? rid : nullptr, &ctx));
    CHECK(pastar_gpu_build_heuristic(ctx));
    if (lead) {
        std::cout << "done!\n";
        std::cout << "Phase 1 - init heuristic: " << mmss(now() - t) << std::endl;
        std::cout << "Performing search with Parallel A-Star.\n";
        std::cout << "Running PAStar with: " << o.threads * o.gpus << " threads (" << o.gpus << " machines with "
                  << o.threads << " threads each)," << kHashName[o.hash_type] << " hash, " << o.hash_shift
                  << " shift.\n";
    }
    pastar_search_opts so{};
    so.batch_nodes = o.batch;
    so.table_slots_log2 = o.table_log2;
    so.pool_entries = o.pool;
    so.verbose = o.verbose;
    t = now();
    CHECK(pastar_gpu_search(ctx, &so, &report->r));
    if (lead)
        std::cout << "Phase 2: PA-Star running time: " << mmss(now() - t) << std::endl;

    int total = 0;
    for (int i = 0; i < n; i++)
        total += lengths[i];
    const int stride = total + 1;
    std::vector<char> rows((size_t)n * stride);
    int cols = 0;
    t = now();
    CHECK(pastar_gpu_alignment(ctx, rows.data(), stride, &cols));
    if (lead) {
        std::cout << "Final Score: (";
        for (int i = 0; i < n; i++)
            std::cout << (i ? " " : "") << lengths[i];
        const long long g = report->r.score;
        std::cout << ")\tg - " << g << " (h - 0 f - " << g << ")" << std::endl;
        std::cout << "Phase 3 - backtrace: " << mmss(now() - t) << std::endl;
        int tot = 0, eq = 0;
        for (int c = 0; c < cols; c++)
            for (int i = 0; i < n; i++)
                for (int j = i + 1; j < n; j++) {
                    eq += rows[(size_t)i * stride + c] == rows[(size_t)j * stride + c];
                    ++tot;
                }
        const float pct = (eq * 100) / (float)tot;
        std::cout << "Similarity: " << std::fixed << std::setprecision(2) << pct << "%" << std::endl;
        const int width = print_width();
        for (int start = 0; start < cols; start += width) {
            std::cout << std::endl;
            for (int i = 0; i < n; i++) {
                const int len = std::min(width, cols - start);
                std::cout.write(&rows[(size_t)i * stride + start], len);
                std::cout << std::endl;
            }
            if (width == INT_MAX)
                break;
        }
        std::cout.flush();
    }
    pastar_gpu_destroy(ctx);
    report->status = 0;
    return 0;
}

// print_nodes_count (PAStar.cpp:591-619), one line per GPU shard.
void print_counts(const std::vector<ShardReport> &reps)
{
    long long open = 0, closed = 0, reopen = 0, total = 0;
    std::cout << "Total nodes count:" << std::endl;
    for (size_t i = 0; i < reps.size(); i++) {
        const pastar_result &r = reps[i].r;
        const long long tot = r.expansions + (i == 0 ? 1 : 0);  // the goal's acceptance
        std::cout << "tid " << i << "\tOpenList:" << r.open_size << "\tClosedList:" << r.closed_size
                  << "\tReopen:" << r.reopen << "\tTotal: " << tot << std::endl;
        open += r.open_size;
        closed += r.closed_size;
        reopen += r.reopen;
        total += tot;
    }
    std::cout << "Sum\tOpenList:" << open << "\tClosedList:" << closed << "\tReopen:" << reopen << "\tTotal: " << total
              << std::endl;
}

}  // namespace

int main(int argc, char **argv)
{
    Options o;
    const int prc = parse(argc, argv, o);
    if (prc != 0)
        return prc < 0 ? 1 : 0;
    if (o.threads <= 0) {  // PAStar.cpp:629-630
        std::cerr << "Running fatal error: Invalid number of threads" << std::endl;
        return 1;
    }
    if (o.hash_shift < 0 || o.hash_shift > 21) {  // CoordHash.cpp:241
        std::cerr << "Running fatal error: Invalid Hash Shift" << std::endl;
        return 1;
    }
    if (o.gpus < 1 || o.gpus > 8) {
        std::cerr << "Invalid argument: --gpus must be 1..8" << std::endl;
        return 1;
    }
    if (o.gpus == 1) {
        std::vector<ShardReport> reps(1);
        if (run_shard(o, 0, nullptr, &reps[0]))
            return 1;
        print_counts(reps);
        return 0;
    }
    // one process per GPU, forked before any HIP call; rank 0 creates the
    // RCCL id and hands it to the others through pipes
    std::vector<int> id_pipe(2 * o.gpus), rep_pipe(2 * o.gpus);
    for (int r = 0; r < o.gpus; r++)
        if (pipe(&id_pipe[2 * r]) || pipe(&rep_pipe[2 * r])) {
            std::perror("pipe");
            return 1;
        }
    std::vector<pid_t> kids;
    for (int r = 0; r < o.gpus; r++) {
        const pid_t pid = fork();
        if (pid < 0) {
            std::perror("fork");
            return 1;
        }
        if (pid == 0) {
            unsigned char rid[128];
            if (r == 0) {
                if (pastar_rccl_unique_id(rid) != PASTAR_OK) {
                    std::cerr << "Running fatal error: " << pastar_last_error() << std::endl;
                    _exit(1);
                }
                for (int k = 1; k < o.gpus; k++)
                    if (write(id_pipe[2 * k + 1], rid, sizeof(rid)) != (ssize_t)sizeof(rid))
                        _exit(1);
            } else if (read(id_pipe[2 * r], rid, sizeof(rid)) != (ssize_t)sizeof(rid)) {
                _exit(1);
            }
            ShardReport rep{};
            rep.status = 1;
            const int rc = run_shard(o, r, rid, &rep);
            if (write(rep_pipe[2 * r + 1], &rep, sizeof(rep)) != (ssize_t)sizeof(rep))
                _exit(1);
            std::cout.flush();
            _exit(rc);
        }
        kids.push_back(pid);
    }
    std::vector<ShardReport> reps(o.gpus);
    int fail = 0;
    for (int r = 0; r < o.gpus; r++) {
        if (read(rep_pipe[2 * r], &reps[r], sizeof(ShardReport)) != (ssize_t)sizeof(ShardReport))
            fail = 1;
    }
    for (pid_t pid : kids) {
        int st = 0;
        waitpid(pid, &st, 0);
        if (!WIFEXITED(st) || WEXITSTATUS(st) != 0)
            fail = 1;
    }
    if (fail)
        return 1;
    print_counts(reps);
    return 0;
}
