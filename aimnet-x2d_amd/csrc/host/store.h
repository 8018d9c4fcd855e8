// The molecule store behind aimx_mol_store handles (include/aimx_host.h), shared by the batch
// builder (collate.cpp) and the HDF5 reader (h5stream.cpp), which fills a store in place instead of
// handing flat arrays to aimx_store_create_hops for one more copy. Internal to the host libraries:
// both are built by the same compiler and libstdc++ (csrc/Makefile).
//
// Invariants every filler keeps (collate reads the store without re-checking them):
// atom_ptr / pair_ptr non-decreasing from 0, n_mols + 1 entries; molecule m's cached pairs are
// pair_ptr[m] .. pair_ptr[m + 1], their hop sizes hop_len[m * cached_hops + h] sum to that count,
// and every local index is < atom_ptr[m + 1] - atom_ptr[m] <= 65535.
#pragma once

#include <cstdint>
#include <vector>

struct aimx_mol_store {
  int64_t n_mols = 0;
  int32_t n_feat = 0, n_tasks = 0, cached_hops = 0;
  std::vector<int64_t> atom_ptr, bond_ptr;
  std::vector<int32_t> bonds, feats;
  std::vector<float> targets, charge;
  // cached hop pairs: pair_ptr[m] .. pair_ptr[m+1] (uint16 (u, w) interleaved, hop-major);
  // hop sizes per molecule in hop_len[m * cached_hops + h]
  std::vector<int64_t> pair_ptr;
  std::vector<uint16_t> pairs;
  std::vector<int32_t> hop_len;
};
