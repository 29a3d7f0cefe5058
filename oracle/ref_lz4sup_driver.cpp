// ref_lz4sup_driver.cpp -- OUR extern "C" wrapper around the reference's own
// pastar/lz4sup.cpp (compiled where it lies under /root/reference by
// oracle/Makefile; nothing is copied), linked against the LZ4 library the
// reference was built with in the survey container (/opt/conda, liblz4
// 1.9.3).  It lets tests/test_wire.py compare the
// engine's wire frames with the reference's byte for byte.
//
// Test infrastructure only; never part of the product, never on the GPU box.
#include <cstring>

#include "include/lz4sup.h"

extern "C" {

// pastar_lz4_en of in[0, len) (in[len] must be the NUL the reference's
// std::string carries); copies the frame to out; returns its size or -1
int ref_lz4_en(const char *in, int len, char *out, int cap)
{
    char *frame = nullptr;
    const int n = pastar_lz4_en(in, &frame, len);
    if (n > cap) {
        delete[] frame;
        return -1;
    }
    std::memcpy(out, frame, (size_t)n);
    delete[] frame;
    return n;
}

// pastar_lz4_dec of a frame; copies the decoded bytes to out; returns their
// count (payload + NUL) or -1
int ref_lz4_dec(const char *frame, int frame_len, char *out, int cap)
{
    char *buf = new char[(size_t)frame_len];
    std::memcpy(buf, frame, (size_t)frame_len);
    const int n = pastar_lz4_dec(&buf);
    if (n > cap) {
        delete[] buf;
        return -1;
    }
    std::memcpy(out, buf, (size_t)n);
    delete[] buf;
    return n;
}
}
