// host_model.cpp -- host-side scoring model (see host_model.hpp).
//
// Build note: compiled with -ffp-contract=off and without fast-math.  The
// Altschul weights are IEEE-single arithmetic whose (int) truncation at use
// (Node.cpp:226, HeuristicHPair.cpp:82) must reproduce the reference bit for
// bit; every float expression below keeps the reference's operation order.
#include "host_model.hpp"

#include <cmath>
#include <cstdio>
#include <cstring>
#include <fstream>

namespace pastar {

// ---------------------------------------------------------------------------
// Distance table (Cost.cpp:12-262), full symmetric matrix in PAM order.
// Entries the reference never assigns are 0: C/S/T against '-' and W-W.
// ---------------------------------------------------------------------------
namespace {
const char kOrder[] = "ARNDCQEGHILKMFPSTWYV-";
const signed char kPam[21][21] = {
    {15, 19, 17, 17, 19, 17, 17, 16, 18, 18, 19, 18, 18, 21, 16, 16, 16, 23, 20, 17, 12},  // A
    {19, 11, 17, 18, 21, 16, 18, 20, 15, 19, 20, 14, 17, 21, 17, 17, 18, 15, 21, 19, 12},  // R
    {17, 17, 15, 15, 21, 16, 16, 17, 15, 19, 20, 16, 19, 21, 18, 16, 17, 21, 19, 19, 12},  // N
    {17, 18, 15, 13, 22, 15, 14, 16, 16, 19, 21, 17, 20, 23, 18, 17, 17, 24, 21, 19, 12},  // D
    {19, 21, 21, 22, 5, 22, 22, 20, 20, 19, 23, 22, 22, 21, 20, 17, 19, 25, 17, 19, 0},    // C
    {17, 16, 16, 15, 22, 13, 15, 18, 14, 19, 19, 16, 18, 22, 17, 18, 18, 22, 21, 19, 12},  // Q
    {17, 18, 16, 14, 22, 15, 13, 17, 16, 19, 20, 17, 19, 22, 18, 17, 17, 24, 21, 19, 12},  // E
    {16, 20, 17, 16, 20, 18, 17, 12, 19, 20, 21, 19, 20, 22, 18, 16, 17, 24, 22, 18, 12},  // G
    {18, 15, 15, 16, 20, 14, 16, 19, 11, 19, 19, 17, 19, 19, 17, 18, 18, 20, 17, 19, 12},  // H
    {18, 19, 19, 19, 19, 19, 19, 20, 19, 12, 15, 19, 15, 16, 19, 18, 17, 22, 18, 13, 12},  // I
    {19, 20, 20, 21, 23, 19, 20, 21, 19, 15, 11, 20, 13, 15, 20, 20, 19, 19, 18, 15, 12},  // L
    {18, 14, 16, 17, 22, 16, 17, 19, 17, 19, 20, 12, 17, 22, 18, 17, 17, 20, 21, 19, 12},  // K
    {18, 17, 19, 20, 22, 18, 19, 20, 19, 15, 13, 17, 11, 17, 19, 19, 18, 21, 19, 15, 12},  // M
    {21, 21, 21, 23, 21, 22, 22, 22, 19, 16, 15, 22, 17, 8, 22, 20, 20, 17, 10, 18, 12},   // F
    {16, 17, 18, 18, 20, 17, 18, 18, 17, 19, 20, 18, 19, 22, 11, 16, 17, 23, 22, 18, 12},  // P
    {16, 17, 16, 17, 17, 18, 17, 16, 18, 18, 20, 17, 19, 20, 16, 15, 16, 19, 20, 18, 0},   // S
    {16, 18, 17, 17, 19, 18, 17, 17, 18, 17, 19, 17, 18, 20, 17, 16, 14, 22, 20, 17, 0},   // T
    {23, 15, 21, 24, 25, 22, 24, 24, 20, 22, 19, 20, 21, 17, 23, 19, 22, 0, 17, 23, 12},   // W
    {20, 21, 19, 21, 17, 21, 21, 22, 17, 18, 18, 21, 19, 10, 22, 20, 20, 17, 7, 19, 12},   // Y
    {17, 19, 19, 19, 19, 19, 19, 18, 19, 13, 15, 19, 15, 18, 18, 18, 17, 23, 19, 13, 12},  // V
    {12, 12, 12, 12, 0, 12, 12, 12, 12, 12, 12, 12, 12, 12, 12, 0, 0, 12, 12, 12, 0},      // -
};

struct Table {
    int v[128][128];
    Table()
    {
        std::memset(v, 0, sizeof(v));
        for (int i = 0; i < 21; i++)
            for (int j = 0; j < 21; j++)
                v[(unsigned char)kOrder[i]][(unsigned char)kOrder[j]] = kPam[i][j];
    }
};
const Table &table()
{
    static const Table t;
    return t;
}
}  // namespace

int ref_cost(int r, int l)
{
    if (r < 0 || l < 0 || r >= 90 || l >= 90)
        return 0;
    return table().v[r][l];
}

// ---------------------------------------------------------------------------
// FASTA (read_fasta.cpp:8-36)
// ---------------------------------------------------------------------------
bool read_fasta(const std::string &path, std::vector<std::string> &seqs)
{
    std::ifstream in(path, std::ios::binary);
    if (!in.is_open())
        return false;
    std::string cur, line;
    while (std::getline(in, line)) {
        if (line.empty() || line[0] == '>') {
            if (!cur.empty())
                seqs.push_back(cur);
            cur.clear();
            continue;
        }
        cur += line;
    }
    if (!cur.empty())
        seqs.push_back(cur);
    return true;
}

// ---------------------------------------------------------------------------
// Altschul rationale-2 weights (WeightedSP.cpp:109-519)
// ---------------------------------------------------------------------------
namespace {

constexpr int kBig = 999999;   // BIG (WeightedSP.hpp:11)
constexpr int kGap = 8;        // GapCost (:17)
constexpr int kEndGap = 0;     // EfectiveGapCost (:21)
constexpr int kInternal = -1;  // INTERNAL_NODE
constexpr int kRoot = -2;      // TREE_ROOT

inline int min_of3(int a, int b, int c)
{
    if (a < b)
        return a < c ? a : c;
    return b < c ? b : c;
}

// Pairwise distance of two '-'-prefixed sequences (primer, :144-244, and
// convert_path_to_cost, :109-142).  End gaps are free; the distance is the
// per-mille mismatch rate of one optimal path, floored at 1.
class Primer {
   public:
    explicit Primer(size_t maxlen) : w_(maxlen), dd_(maxlen * maxlen), hh_(dd_.size()), vv_(dd_.size()) {}

    int distance(const std::string &A, const std::string &B)
    {
        const int n = (int)A.size(), m = (int)B.size();
        D(0, 0) = 0;
        H(0, 0) = V(0, 0) = kEndGap;
        for (int j = 1; j < m; j++) {
            V(0, j) = D(0, j) = kBig;
            H(0, j) = H(0, j - 1) + ref_cost('-', B[j]);
        }
        for (int i = 1; i < n; i++) {
            H(i, 0) = D(i, 0) = kBig;
            V(i, 0) = V(i - 1, 0) + ref_cost(A[i], '-');
        }
        for (int i = 1; i < n; i++) {
            const int gi = (i == n - 1) ? kEndGap : kGap;
            for (int j = 1; j < m; j++) {
                const int gj = (j == m - 1) ? kEndGap : kGap;
                D(i, j) = min_of3(D(i - 1, j - 1), H(i - 1, j - 1), V(i - 1, j - 1)) + ref_cost(A[i], B[j]);
                H(i, j) = min_of3(D(i, j - 1) + gi, H(i, j - 1), V(i, j - 1) + gi) + ref_cost('-', B[j]);
                V(i, j) = min_of3(D(i - 1, j) + gj, H(i - 1, j) + gj, V(i - 1, j)) + ref_cost(A[i], '-');
            }
        }
        // traceback from (n-1, m-1) counting identical aligned residues
        const int nn = n - 1, mm = m - 1;
        enum { Diag, Vert, Horz } dir = Diag;
        int match = 0;
        for (int i = nn, j = mm; i || j;) {
            const int v = V(i, j) - (dir == Vert ? (j == mm ? kEndGap : kGap) : 0);
            const int h = H(i, j) - (dir == Horz ? (i == nn ? kEndGap : kGap) : 0);
            const int best = min_of3(v, h, D(i, j));
            if (!j || best == v) {
                dir = Vert;
                --i;
            } else if (!i || best == h) {
                dir = Horz;
                --j;
            } else {
                dir = Diag;
                match += A[i] == B[j];
                --i;
                --j;
            }
        }
        return (int)(0.5 + 1000.0 * (nn - match + mm - match) / (nn + mm));
    }

   private:
    int &D(int i, int j) { return dd_[(size_t)i * w_ + j]; }
    int &H(int i, int j) { return hh_[(size_t)i * w_ + j]; }
    int &V(int i, int j) { return vv_[(size_t)i * w_ + j]; }
    size_t w_;
    std::vector<int> dd_, hh_, vv_;
};

// Neighbour-joining tree over the leaves (phylogeneticThreeNeighborJoin,
// :317-401) and Altschul's partial weights on it (:455-495).
class Tree {
   public:
    struct Node {
        int parent = -1, left = -1, right = -1, brother = -1;
        float weight = 0.0f, w = 0.0f, W = 0.0f, v = 0.0f, V = 0.0f;
        int seq = kInternal;
    };

    Tree(int n, const std::vector<float> &dist) : n_(n), dist_(dist) {}

    void build()
    {
        std::vector<int> live;
        for (int i = 0; i < n_; i++) {
            live.push_back(add(-1, -1, i));
            order_.push_back(live.back());
        }
        while ((int)live.size() > 2) {
            const int k = (int)live.size();
            float best = (float)1.0E20;
            int bi = 0, bj = 0;
            for (int i = 0; i < k - 1; i++)
                for (int j = i + 1; j < k; j++) {
                    const float s = join_score(live, i, j);
                    if (s < best) {
                        bi = i;
                        bj = j;
                        best = s;
                    }
                }
            join(live, bi, bj);
        }
        const int l = live[0], r = live[1];
        const int root = add(l, r, kRoot);
        link(l, r, root);
        order_.push_back(root);
        int c = 1;
        float len = path_cost(l, r);
        float t = leaf_depth(l, 0.0f, &c);
        len -= t / c;
        c = 1;
        t = leaf_depth(r, 0.0f, &c);
        len -= t / c;
        nodes_[l].weight = len;
    }

    // rationale-2 pair weights, unscaled: out[x*n+y] for every x != y
    void pair_weights(std::vector<float> &out)
    {
        size_t p = 0;
        for (; nodes_[order_[p]].seq > kInternal; ++p) {
            Node &a = nodes_[order_[p]];
            a.w = 1.0f;
            a.W = a.weight;
        }
        for (; nodes_[order_[p]].seq > kRoot; ++p) {
            Node &a = nodes_[order_[p]];
            const Node &l = nodes_[a.left], &r = nodes_[a.right];
            a.w = l.w * r.W + l.W * r.w;
            a.W = a.weight * a.w + l.W * r.W;
        }
        nodes_[order_[p]].V = 1;
        nodes_[order_[p]].v = 0;
        do {
            Node &a = nodes_[order_[--p]];
            const Node &pa = nodes_[a.parent], &br = nodes_[a.brother];
            a.v = pa.v * br.W + pa.V * br.w;
            a.V = a.weight * a.v + pa.V * br.W;
        } while (p != 0);
        out.assign((size_t)n_ * n_, 0.0f);
        for (; nodes_[order_[p]].seq > kInternal; ++p) {
            const Node &a = nodes_[order_[p]];
            walk(out, a.seq, 1.0f, a.weight, a.parent, a.brother);
        }
    }

   private:
    int add(int l, int r, int seq)
    {
        Node x;
        x.left = l;
        x.right = r;
        x.seq = seq;
        nodes_.push_back(x);
        return (int)nodes_.size() - 1;
    }
    void link(int l, int r, int parent)
    {
        nodes_[l].brother = r;
        nodes_[r].brother = l;
        nodes_[l].parent = nodes_[r].parent = parent;
    }
    // compute_path_cost_rec (:249-264): sum of leaf distances across the two
    // subtrees, counting the internal nodes crossed.
    float path_sum(int a, int b, int *len) const
    {
        if (nodes_[a].seq < 0) {
            ++*len;
            return path_sum(nodes_[a].left, b, len) + path_sum(nodes_[a].right, b, len);
        }
        if (nodes_[b].seq < 0) {
            ++*len;
            return path_sum(a, nodes_[b].left, len) + path_sum(a, nodes_[b].right, len);
        }
        return dist_[(size_t)nodes_[a].seq * n_ + nodes_[b].seq];
    }
    float path_cost(int a, int b) const  // compute_path_cost (:268-275)
    {
        int len = 1;
        const float s = path_sum(a, b, &len);
        return (float)(s / len);
    }
    // compute_path_cost_to_leafs (:56-62)
    float leaf_depth(int a, float total, int *count) const
    {
        const Node &x = nodes_[a];
        if (x.seq >= 0)
            return total + x.weight;
        (*count)++;
        return leaf_depth(x.left, x.weight + total, count) + leaf_depth(x.right, x.weight + total, count);
    }
    // compute_S (:287-309)
    float join_score(const std::vector<int> &live, int i, int j) const
    {
        const int k = (int)live.size();
        float s1 = 0, s2 = 0;
        for (int t = 0; t < k; t++)
            if (t != i && t != j)
                s1 += path_cost(live[i], live[t]) + path_cost(live[j], live[t]);
        s1 = s1 / (2 * (k - 2));
        for (int t = 0; t < k - 1; t++)
            for (int u = t + 1; u < k; u++)
                if (t != i && t != j && u != i && u != j)
                    s2 += path_cost(live[t], live[u]);
        s2 = s2 / (k - 2);
        return (s1 + s2 + path_cost(live[i], live[j]) / 2);
    }
    // compute_curr_cost (:64-76): branch length of live[i] when joined to
    // live[j]; the leaf-depth divisor is read after the walk that bumps it.
    float branch(const std::vector<int> &live, int i, int j) const
    {
        const int k = (int)live.size();
        float di = 0.0f, dj = 0.0f;
        int c = 1;
        for (int t = 0; t < k; ++t)
            if (t != i && t != j) {
                di += path_cost(live[i], live[t]);
                dj += path_cost(live[j], live[t]);
            }
        di = di / (k - 2);
        dj = dj / (k - 2);
        const float head = (path_cost(live[i], live[j]) + di - dj) / 2;
        const float depth = leaf_depth(live[i], 0.0f, &c);
        return head - depth / c;
    }
    // join_nodes (:78-107)
    void join(std::vector<int> &live, int i, int j)
    {
        const int l = live[i];
        nodes_[l].weight = branch(live, i, j);
        const int r = live[j];
        nodes_[r].weight = branch(live, j, i);
        const int x = add(l, r, kInternal);
        link(l, r, x);
        order_.push_back(x);
        live[i] = x;
        live[j] = live.back();
        live.pop_back();
    }
    // compute_weights_from_tree (:405-421)
    void walk(std::vector<float> &out, int leaf, float product, float sum, int at, int brother) const
    {
        const Node &x = nodes_[at];
        if (x.seq > kInternal) {
            out[(size_t)leaf * n_ + x.seq] = sum * product;
        } else if (brother < 0) {
            walk(out, leaf, product * nodes_[x.left].W, sum + nodes_[x.right].weight, x.right, -1);
            walk(out, leaf, product * nodes_[x.right].W, sum + nodes_[x.left].weight, x.left, -1);
        } else {
            walk(out, leaf, product * x.V, sum + nodes_[brother].weight, brother, -1);
            if (x.seq != kRoot)
                walk(out, leaf, product * nodes_[brother].W, sum + x.weight, x.parent, x.brother);
        }
    }

    int n_;
    const std::vector<float> &dist_;
    std::vector<Node> nodes_;
    std::vector<int> order_;  // nodesList: leaves, joins in order, root
};

}  // namespace

std::vector<float> altschul_weights(const std::vector<std::string> &in)
{
    const int n = (int)in.size();
    std::vector<std::string> seqs;
    size_t maxlen = 1;
    for (const auto &s : in) {
        seqs.push_back("-" + s);  // WeightedSP.cpp:447
        maxlen = std::max(maxlen, seqs.back().size());
    }
    std::vector<float> dist((size_t)n * n, 0.0f);
    Primer primer(maxlen);
    for (int i = 0; i < n - 1; i++)
        for (int j = i + 1; j < n; j++) {
            float d = (float)primer.distance(seqs[i], seqs[j]);
            if (d <= 0)
                d = 1;
            dist[(size_t)i * n + j] = dist[(size_t)j * n + i] = d;
        }
    Tree tree(n, dist);
    tree.build();
    std::vector<float> wm;
    tree.pair_weights(wm);

    float sm = 1.0E+30f;  // scale: smallest pair weight ~ 7.9 (:497-509)
    for (int j = 1; j < n; ++j)
        for (int i = 0; i < j; ++i)
            if (wm[(size_t)i * n + j] < sm)
                sm = wm[(size_t)i * n + j];
    sm = (float)(sm / 7.9);
    std::vector<float> out((size_t)n * n, 0.0f);
    for (int i = 0; i < n - 1; ++i)
        for (int j = i + 1; j < n; ++j) {
            const float q = wm[(size_t)i * n + j] / sm;
            out[(size_t)i * n + j] = out[(size_t)j * n + i] = (float)((double)q + 0.5);
        }
    return out;
}

// ---------------------------------------------------------------------------
// CoordHash (CoordHash.cpp:28-245)
// ---------------------------------------------------------------------------
namespace {
// z_order_hash<Shift> (:107-134) over `dims` coordinates; PZORDER is dims 2.
unsigned zorder(int dims, const uint16_t *c, int size, int shift)
{
    int hash = 0;
    int bit_to_read = shift / dims;
    const unsigned bits = (unsigned)(std::log2((double)size) + (shift % dims) + 1);
    const unsigned total = bits >= 31 ? 0x80000000u : (1u << bits);
    for (unsigned bit = 1; bit != 0 && bit <= total;) {
        for (int j = 0; j < dims && bit != 0 && bit <= total; ++j) {
            if (bit_to_read < 16 && (c[j] & (1u << bit_to_read)))
                hash = (int)((unsigned)hash | bit);
            bit <<= 1;
        }
        ++bit_to_read;
    }
    return (unsigned)((hash >> (shift % dims)) % size);
}
}  // namespace

int owner_of(int n, const uint16_t *c, int size, int hash_type, int shift)
{
    if (shift < 0 || shift > 21 || size <= 0 || n < 2)
        return -1;
    switch (hash_type) {
    case 2: {  // HashFSum
        unsigned s = 0;
        for (int i = 0; i < n; i++)
            s += c[i];
        return (int)((s >> shift) % (unsigned)size);
    }
    case 3:  // HashPSum
        return (int)(((unsigned)(c[0] + c[1]) >> shift) % (unsigned)size);
    case 1:  // HashPZorder
        return (int)zorder(2, c, size, shift);
    case 0:  // HashFZorder
        return (int)zorder(n, c, size, shift);
    default:
        return -1;
    }
}

}  // namespace pastar
