// Device restatement of numpy's float64 add.reduce (pairwise summation) so that
// np.sum / np.mean / np.std over the same float64 inputs give the same bits on
// the GPU.  numpy: DOUBLE_pairwise_sum (numpy/_core/src/umath/loops_utils.h.src):
//   n < 8      : res = -0.0; res += a[i] ...
//   n <= 128   : 8 interleaved accumulators, ((r0+r1)+(r2+r3))+((r4+r5)+(r6+r7)), tail
//   otherwise  : n2 = n/2 - (n/2)%8; sum(a, n2) + sum(a+n2, n-n2)
// np.add.reduce(a) starts from the identity 0.0 and adds the pairwise sum of each
// 8192-element buffer chunk in turn (the ufunc reduction's buffer size):
//   s = 0.0; for each chunk: s += pairwise(chunk)     (checked on numpy 2.2, n <= 432000)
// mean = sum/n; std = sqrt(sum((a-mean)^2)/n) (population, numpy _var).
// FP contraction is switched off inside every function here (no FMA may fuse a
// multiply numpy rounds separately).
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>

namespace msd {

// A(i) returns the i-th element (a functor, so (x-mean)^2 can be formed on the fly
// exactly as numpy materialises it: one rounded subtract, one rounded multiply).
template <typename A>
__device__ __forceinline__ double np_pairwise_leaf(const A &a, int64_t base, int64_t n) {
#pragma clang fp contract(off)
    if (n < 8) {
        double res = -0.0;
        for (int64_t i = 0; i < n; ++i) res += a(base + i);
        return res;
    }
    double r0 = a(base + 0), r1 = a(base + 1), r2 = a(base + 2), r3 = a(base + 3);
    double r4 = a(base + 4), r5 = a(base + 5), r6 = a(base + 6), r7 = a(base + 7);
    int64_t i = 8;
    const int64_t lim = n - (n % 8);
    for (; i < lim; i += 8) {
        r0 += a(base + i + 0);
        r1 += a(base + i + 1);
        r2 += a(base + i + 2);
        r3 += a(base + i + 3);
        r4 += a(base + i + 4);
        r5 += a(base + i + 5);
        r6 += a(base + i + 6);
        r7 += a(base + i + 7);
    }
    double res = ((r0 + r1) + (r2 + r3)) + ((r4 + r5) + (r6 + r7));
    for (; i < n; ++i) res += a(base + i);
    return res;
}

// numpy's recursion tree over [base, base+n) walked iteratively, for n <= NP_ITER_MAX[DMAX] (tree
// depth <= DMAX): the leaves in order (leaf(b, m) returns a leaf's sum, m <= 128), the pending right
// subtrees and the finished left sums on register stacks that are shifted, never indexed (no
// scratch), each internal node combined as left + right (numpy's association).  Every lane runs the
// same loop and one copy of the leaf code, so a wave whose lanes sum ranges of different lengths runs
// the leaves in lockstep; the recursion inlined one leaf copy per tree shape (128 at depth 7: the
// 100-180 KB np_pairwise functions), which the lanes of such a wave ran one after another.
constexpr int NP_ITER_MAX[8] = {128, 248, 488, 968, 1928, 3848, 7688, 8192};  // largest n of depth <= D

template <int DMAX, typename LeafFn>
__device__ __forceinline__ double np_walk_iter(int64_t base, int n, const LeafFn &leaf) {
#pragma clang fp contract(off)
    int pb[DMAX], ps[DMAX];  // pending right subtrees (offset, size), top = [0]
    double pv[DMAX];         // left-subtree sums waiting for their right sibling, top = [0]
#pragma unroll
    for (int k = 0; k < DMAX; ++k) pb[k] = ps[k] = 0, pv[k] = 0.0;
    int b = 0, s = n, d = 0;
    unsigned right = 0;  // bit d: the node at depth d is a right child
    for (;;) {
        while (s > 128) {  // down to the leftmost leaf, the right halves pending
            int s2 = s / 2;
            s2 -= s2 % 8;
#pragma unroll
            for (int k = DMAX - 1; k > 0; --k) pb[k] = pb[k - 1], ps[k] = ps[k - 1];
            pb[0] = b + s2;
            ps[0] = s - s2;
            s = s2;
            ++d;
            right &= ~(1u << d);
        }
        double v = leaf(base + b, (int64_t)s);
        while (d > 0 && ((right >> d) & 1u)) {  // a right subtree done: its parent = left + right
            v = pv[0] + v;
#pragma unroll
            for (int k = 0; k < DMAX - 1; ++k) pv[k] = pv[k + 1];
            --d;
        }
        if (d == 0) return v;
#pragma unroll
        for (int k = DMAX - 1; k > 0; --k) pv[k] = pv[k - 1];
        pv[0] = v;  // a left subtree done: on to its right sibling
        b = pb[0];
        s = ps[0];
#pragma unroll
        for (int k = 0; k < DMAX - 1; ++k) pb[k] = pb[k + 1], ps[k] = ps[k + 1];
        right |= 1u << d;
    }
}

template <int DMAX, typename A>
__device__ __forceinline__ double np_pairwise_iter(const A &a, int64_t base, int n) {
    return np_walk_iter<DMAX>(base, n, [&](int64_t b, int64_t m) { return np_pairwise_leaf(a, b, m); });
}

// numpy's recursion tree over one ufunc buffer chunk (n <= 8192), leaves in order (left subtree
// first), combined as numpy's recursion does.  An earlier iterative form kept its stack in an
// indexed array, i.e. in scratch (1.2 KB per lane in detect.hip's leaf-table builder); the
// compile-time recursion that replaced it inlined one leaf copy per tree shape.  np_walk_iter has
// neither problem.
template <typename LeafFn>
__device__ double np_tree_walk(int64_t base, int64_t n, const LeafFn &leaf) {
    return np_walk_iter<7>(base, (int)n, leaf);
}

// numpy's recursion written as compile-time recursion over the depth (n <= 8192 needs at most 7
// splits): for a shallow, known depth (stream.hip's canonical blocks, D = 2)
template <int D, typename A>
__device__ __forceinline__ double np_pairwise_rec(const A &a, int64_t base, int64_t n) {
#pragma clang fp contract(off)
    if constexpr (D == 0) {
        return np_pairwise_leaf(a, base, n);
    } else {
        if (n <= 128) return np_pairwise_leaf(a, base, n);
        int64_t n2 = n / 2;
        n2 -= n2 % 8;
        const double l = np_pairwise_rec<D - 1>(a, base, n2);
        return l + np_pairwise_rec<D - 1>(a, base + n2, n - n2);
    }
}

template <typename A>
__device__ double np_pairwise(const A &a, int64_t base, int64_t n) {  // n <= NP_BUFSIZE
    return np_pairwise_iter<7>(a, base, (int)n);
}

constexpr int64_t NP_BUFSIZE = 8192;

template <typename A>
__device__ double np_sum(const A &a, int64_t base, int64_t n) {
#pragma clang fp contract(off)
    double s = 0.0;
    for (int64_t c = 0; c < n; c += NP_BUFSIZE) s += np_pairwise(a, base + c, n - c < NP_BUFSIZE ? n - c : NP_BUFSIZE);
    return s;
}

// np.sum for n <= 128 (a single pairwise leaf; no recursion stack)
template <typename A>
__device__ __forceinline__ double np_sum_small(const A &a, int64_t base, int64_t n) {
#pragma clang fp contract(off)
    return n == 0 ? 0.0 : 0.0 + np_pairwise_leaf(a, base, n);
}

struct ArrRef {
    const double *p;
    __device__ double operator()(int64_t i) const { return p[i]; }
};
struct SqDevRef {
    const double *p;
    double mean;
    __device__ double operator()(int64_t i) const {
#pragma clang fp contract(off)
        const double d = p[i] - mean;
        return d * d;
    }
};

// Global memory typed as such (address space 1), for data read by out-of-line device functions.  A
// pointer that reaches a callee is generic, and generic loads are flat instructions, which pick LDS,
// scratch or global from the high bits of the address register alone -- the instruction's offset is
// not looked at.  A loop pointer the compiler displaces below an LDS object (base - 64 with offsets
// +128 ..) therefore leaves the LDS aperture: round 5's one GPU fault.  Out-of-line
// code reads global data through these (global_load) and never receives an LDS pointer;
// tests/test_build_check.py holds every function of the library to zero flat instructions.
typedef const __attribute__((address_space(1))) double gdouble_t;
__device__ __forceinline__ gdouble_t *as_global(const double *p) { return (gdouble_t *)p; }
struct GArrRef {
    gdouble_t *p;
    __device__ double operator()(int64_t i) const { return p[i]; }
};
struct GSqDevRef {
    gdouble_t *p;
    double mean;
    __device__ double operator()(int64_t i) const {
#pragma clang fp contract(off)
        const double d = p[i] - mean;
        return d * d;
    }
};

// numpy mean/std of p[base .. base+n), n <= NP_ITER_MAX[DMAX], by np_pairwise_iter
template <int DMAX>
__device__ __forceinline__ void np_mean_std_iter(const double *p, int64_t base, int n, double &mean, double &std) {
#pragma clang fp contract(off)
    const double s = 0.0 + np_pairwise_iter<DMAX>(ArrRef{p}, base, n);
    mean = s / (double)n;
    const double v = 0.0 + np_pairwise_iter<DMAX>(SqDevRef{p, mean}, base, n);
    std = sqrt(v / (double)n);
}

// numpy mean/std of p[base .. base+n).  n <= 128 (one pairwise leaf) stays inline: the general
// np_sum is a large out-of-line function whose call and instruction-cache misses cost more
// than the sum itself in the event handlers of the live scan (live.hip)
// numpy mean/std of global p[base .. base+n) through global loads (GArrRef): for out-of-line callers
__device__ __forceinline__ void np_mean_std_global(const double *p, int64_t base, int64_t n, double &mean,
                                                   double &std) {
#pragma clang fp contract(off)
    const GArrRef a{as_global(p)};
    const double s = n <= 128 ? np_sum_small(a, base, n) : np_sum(a, base, n);
    mean = s / (double)n;
    const GSqDevRef q{a.p, mean};
    const double v = n <= 128 ? np_sum_small(q, base, n) : np_sum(q, base, n);
    std = sqrt(v / (double)n);
}

__device__ __forceinline__ void np_mean_std(const double *p, int64_t base, int64_t n, double &mean, double &std) {
#pragma clang fp contract(off)
    if (n <= 128) {
        const double s = np_sum_small(ArrRef{p}, base, n);
        mean = s / (double)n;
        const double v = np_sum_small(SqDevRef{p, mean}, base, n);
        std = sqrt(v / (double)n);
        return;
    }
    const double s = np_sum(ArrRef{p}, base, n);
    mean = s / (double)n;
    const double v = np_sum(SqDevRef{p, mean}, base, n);
    std = sqrt(v / (double)n);
}

}  // namespace msd
