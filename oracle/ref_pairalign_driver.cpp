// ref_pairalign_driver.cpp -- OUR driver around the reference's own
// pastar/Cost.cpp and pastar/PairAlign.cpp (compiled where they lie under
// /root/reference by oracle/Makefile; nothing is copied).  Those two files
// need no Boost, so this is the one slice of the reference that builds here.
//
//   ref_pairalign SEQ1 SEQ2   -> prints "l1 l2" then the (l1+1)*(l2+1) table
//                                of PairAlign::getScore(i, j), row-major
//   ref_pairalign --cost      -> prints the 128x128 Cost::cost(r, l) table for
//                                r, l in 0..89 (the reference's array bounds)
//
// Test infrastructure only (tests/test_oracle.py); never part of the product.
#include <cstdio>
#include <cstring>
#include <string>

#include "include/Cost.h"
#include "include/PairAlign.h"

int main(int argc, char **argv)
{
    if (argc == 2 && !strcmp(argv[1], "--cost")) {
        for (int r = 0; r < 90; r++) {
            for (int l = 0; l < 90; l++)
                printf("%d%c", Cost::cost((char)r, (char)l), l == 89 ? '\n' : ' ');
        }
        return 0;
    }
    if (argc != 3) {
        fprintf(stderr, "usage: %s SEQ1 SEQ2 | --cost\n", argv[0]);
        return 2;
    }
    std::string a(argv[1]), b(argv[2]);
    PairAlign pa(Pair(0, 1), a, b);
    printf("%zu %zu\n", a.size(), b.size());
    for (size_t i = 0; i <= a.size(); i++) {
        for (size_t j = 0; j <= b.size(); j++)
            printf("%d%c", pa.getScore((int)i, (int)j), j == b.size() ? '\n' : ' ');
    }
    return 0;
}
