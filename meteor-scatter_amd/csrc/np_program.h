// numpy's np.sum association over n elements as a list of leaf records (plain C++, no HIP):
// add.reduce over a contiguous float64 array is s = 0.0; s += pairwise(chunk) over 8192-element
// chunks in order, and pairwise(m) splits m > 128 at n2 = m/2 - (m/2 % 8) (numpy
// pairwise_sum, loops_utils.h.src).  One record per leaf of <= 128 elements, in order:
// {offset, length, adds that follow it (each combines the two top partial sums), 1 if a chunk
// ends after them (s += its sum)}.  stream.hip's fresh_kernel runs the records; host_check.cpp
// checks them under the sanitizers.
#pragma once

#include <cstdint>
#include <vector>

namespace msd {

struct LeafRec {  // layout of HIP's int4 (the device copy is a memcpy of the vector)
    int off, len, adds, chunk_end;
};

constexpr int64_t NP_CHUNK = 8192;

inline void np_tree_records(int64_t base, int64_t m, std::vector<LeafRec> &r) {
    if (m <= 128) {
        r.push_back(LeafRec{(int)base, (int)m, 0, 0});
        return;
    }
    int64_t m2 = m / 2;
    m2 -= m2 % 8;
    np_tree_records(base, m2, r);
    np_tree_records(base + m2, m - m2, r);
    r.back().adds += 1;  // the add combining the two halves follows the right half's last leaf
}

inline void build_program(int64_t n, std::vector<LeafRec> &rec) {
    rec.clear();
    for (int64_t c = 0; c < n; c += NP_CHUNK) {
        const int64_t m = n - c < NP_CHUNK ? n - c : NP_CHUNK;
        np_tree_records(c, m, rec);
        rec.back().chunk_end = 1;
    }
}

}  // namespace msd
