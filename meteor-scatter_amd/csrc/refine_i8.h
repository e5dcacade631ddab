// The int8-MFMA block step of msd_iq_delta64_dev (refine_i8.hip): exact integer DFTs of int16 I/Q
// blocks at the needed bins, written as refine.hip's bin-major block table.
#pragma once

#include "msd_internal.h"
#include "refine_plan.h"

namespace msd {

// D = 1024 blocks, no bin 0 among the needed ones (the detrend then only zeroes it), <= 10 bins
bool i8_supported(const RefineGeom &G, const RefineBins &K);
// blk: [nk + 2][nblocks] double2 as block_kernel writes it; asynchronous on ctx->stream
int launch_refine_i8(msd_ctx *ctx, const int16_t *x, const RefineGeom &G, const RefineBins &K, const int64_t *d_bstart,
                     const int64_t *d_bcs, int64_t nblocks, double2 *blk);
// our own rounding chain (units of u = 2^-53) up to the block values, as RefineGeom::chain's `own`
double i8_chain_own();

}  // namespace msd
