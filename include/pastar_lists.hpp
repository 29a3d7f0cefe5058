// pastar_lists.hpp -- the reference's OpenList and ClosedList classes over the
// C-ABI of include/pastar_gpu.h, for C++ callers of the drop-in.
//
//   reference                                    here
//   -------------------------------------------  ------------------------------
//   PriorityList<N> (PriorityList.h:52-122)      pastar::PriorityList<N>
//     dequeue, conditional_enqueue,                same names and return
//     get_highest_priority, find, erase,           values; the list lives on
//     size, empty                                  the device (pastar_gpu_open_*)
//   ClosedList[tid] std::map (PAStar.cpp:92)     pastar::ClosedList<N>
//     find, erase, size                            (pastar_gpu_lists_*)
//   PAStar::enqueue (PAStar.cpp:219-237)         PriorityList::enqueue(vector)
//
// Two deviations from the reference's classes, both forced by one device node
// record serving both lists (see pastar_gpu.h):
//  - dequeue moves its node into the ClosedList (worker_inner's
//    `ClosedList[pos] = current`, PAStar.cpp:351, which can never refuse a
//    node the OpenList just gave up);
//  - conditional_enqueue includes PAStar::enqueue's ClosedList check
//    (PAStar.cpp:226-232): a node that sits in the ClosedList with g <= the
//    new g is discarded, one with a larger g leaves the ClosedList (a
//    reopening).  The reference's PriorityList alone would hold such a node
//    in both lists; the reference never asks it to: each of its calls of
//    conditional_enqueue comes behind that check or an erase (PAStar.cpp:
//    226-234, 531-537; AStar.cpp:86-93).
// Errors throw pastar::Error with the C-ABI status and message.
#ifndef PASTAR_LISTS_HPP
#define PASTAR_LISTS_HPP

#include <cstdint>
#include <stdexcept>
#include <string>
#include <vector>

#include "pastar_gpu.h"

namespace pastar {

class Error : public std::runtime_error {
   public:
    explicit Error(int code_)
        : std::runtime_error(std::string(pastar_last_error()) + " (status " + std::to_string(code_) + ")"), code(code_)
    {
    }
    int code;
};

inline void check(int rc)
{
    if (rc != PASTAR_OK)
        throw Error(rc);
}

template <int N>
class PriorityList {
    static_assert(N >= 2 && N <= PASTAR_MAX_SEQ, "2..PASTAR_MAX_SEQ sequences");

   public:
    // an empty OpenList + ClosedList pair on the context (PAStar's lists)
    explicit PriorityList(pastar_ctx *ctx, const pastar_search_opts *opts = nullptr) : ctx_(ctx)
    {
        check(pastar_gpu_lists_reset(ctx, opts));
    }

    // the lowest-f node (PriorityList.h:84-93); false when empty
    bool dequeue(pastar_node &n)
    {
        int cnt = 0;
        check(pastar_gpu_open_dequeue(ctx_, &n, 1, &cnt));
        return cnt == 1;
    }

    // up to max nodes, all of the lowest f
    int dequeue(std::vector<pastar_node> &out, int max)
    {
        out.resize((size_t)max);
        int cnt = 0;
        check(pastar_gpu_open_dequeue(ctx_, out.data(), max, &cnt));
        out.resize((size_t)cnt);
        return cnt;
    }

    // PriorityList.h:104-113.  Returns what the reference returns: true
    // whether n was inserted, replaced a worse record, or was discarded as
    // not better (:109-110 returns true for that too; insert and modify
    // cannot fail there).  *entered (optional) tells the cases apart: true
    // when n is now the OpenList's record of its coordinate.
    bool conditional_enqueue(const pastar_node &n, bool *entered = nullptr)
    {
        int32_t added = 0;
        check(pastar_gpu_open_enqueue(ctx_, &n, 1, &added, nullptr));
        if (entered)
            *entered = added != 0;
        return true;
    }

    // PAStar::enqueue (PAStar.cpp:219-237) over a batch; returns the nodes
    // reopened (taken back from the ClosedList with a smaller g)
    int64_t enqueue(const std::vector<pastar_node> &nodes)
    {
        int64_t reopened = 0;
        if (!nodes.empty())
            check(pastar_gpu_open_enqueue(ctx_, nodes.data(), (int)nodes.size(), nullptr, &reopened));
        return reopened;
    }

    // PriorityList.h:116-122: INT_MAX when empty
    int get_highest_priority() const
    {
        int32_t f = 0;
        check(pastar_gpu_open_highest_priority(ctx_, &f));
        return f;
    }

    size_t size() const
    {
        int64_t open = 0, closed = 0;
        check(pastar_gpu_lists_size(ctx_, &open, &closed));
        return (size_t)open;
    }

    bool empty() const { return get_highest_priority() == INT32_MAX; }

    bool find(const uint16_t *pos, pastar_node *out = nullptr) const
    {
        int where = 0;
        check(pastar_gpu_lists_find(ctx_, pos, out, &where));
        return where == 1;
    }

    size_t erase(const uint16_t *pos)
    {
        int erased = 0;
        check(pastar_gpu_lists_erase(ctx_, pos, 1, &erased));
        return (size_t)erased;
    }

    int64_t reopened() const
    {
        int64_t r = 0;
        check(pastar_gpu_lists_reopened(ctx_, &r));
        return r;
    }

   private:
    pastar_ctx *ctx_;
};

template <int N>
class ClosedList {
   public:
    explicit ClosedList(pastar_ctx *ctx) : ctx_(ctx) {}

    bool find(const uint16_t *pos, pastar_node *out = nullptr) const
    {
        int where = 0;
        check(pastar_gpu_lists_find(ctx_, pos, out, &where));
        return where == 2;
    }

    size_t erase(const uint16_t *pos)
    {
        int erased = 0;
        check(pastar_gpu_lists_erase(ctx_, pos, 2, &erased));
        return (size_t)erased;
    }

    size_t size() const
    {
        int64_t open = 0, closed = 0;
        check(pastar_gpu_lists_size(ctx_, &open, &closed));
        return (size_t)closed;
    }

   private:
    pastar_ctx *ctx_;
};

}  // namespace pastar

#endif
