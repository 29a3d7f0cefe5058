// host_model.hpp -- host-side scoring model of the PAStar engine: FASTA input,
// the reference distance table, Altschul rationale-2 pair weights and the
// CoordHash owner function.  All of it is one-off host precompute in the
// reference too; the search itself runs on the GPU.
#pragma once

#include <cstdint>
#include <string>
#include <vector>

namespace pastar {

constexpr int kMaxSeq = 16;

// Cost::cost (Cost.cpp:266-270) on the reference table.  Residues outside the
// reference's int[90][90] (index >= 90: 'Z', lowercase, bytes >= 0x80) read
// out of bounds there; they cost 0 here (see DESIGN.md "Cost quirks").
int ref_cost(int r, int l);

// read_fasta_file_core (read_fasta.cpp:8-36).  Returns false if unreadable.
bool read_fasta(const std::string &path, std::vector<std::string> &seqs);

// weightAltschulsRationale2 (WeightedSP.cpp:424-519): returns the n*n float
// matrix the reference stores in HeuristicHPair::weightMatrix.
std::vector<float> altschul_weights(const std::vector<std::string> &seqs);

// Coord<N>::get_id (CoordHash.cpp:191-245).  -1 for an invalid shift.
int owner_of(int n, const uint16_t *pos, int size, int hash_type, int shift);

}  // namespace pastar
