/* SPDX-License-Identifier: BSD-3-Clause
 *
 * Streaming floors for the classifier's launch shape (diagnostics, not part
 * of the classification path): read npkt 64-byte frames, write one u32 per
 * frame, with the access patterns the classifier could use. DESIGN.md quotes
 * these as the achievable HBM floor of a 2^20-packet batch.
 *
 *   pattern 0  coalesced: consecutive lanes read consecutive 16 B
 *   pattern 1  lane per frame: 4 x 16 B loads per lane (the register fast path)
 *   pattern 2  coalesced 16 B loads into LDS, then lane-per-frame LDS reads
 *   | 0x10     nontemporal loads
 */
#include <hip/hip_runtime.h>
#include <errno.h>
#include <stdint.h>

#include "../../include/odpg.h"

#define DBLOCK 256

typedef unsigned int d_u32x4 __attribute__((ext_vector_type(4)));

template <bool NT>
__device__ __forceinline__ d_u32x4 dld(const d_u32x4 *p)
{
	if (NT)
		return __builtin_nontemporal_load(p);
	return *p;
}

template <int PAT, bool NT>
__global__ __launch_bounds__(DBLOCK) void odpg_diag_stream_kernel(const d_u32x4 *__restrict__ src,
								 uint32_t npkt,
								 uint32_t *__restrict__ out)
{
	__shared__ uint32_t lds[DBLOCK * 17];
	const uint32_t tid = threadIdx.x;
	const uint32_t ntiles = (npkt + DBLOCK - 1) / DBLOCK;

	for (uint32_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
		const uint32_t p0 = tile * DBLOCK;
		uint32_t x = 0u;

		if (PAT == 0) {
			/* 4 lanes per frame, 4 passes of a fully coalesced 4 KiB span */
#pragma unroll
			for (int k = 0; k < 4; ++k) {
				const uint32_t q = k * DBLOCK + tid;          /* 16-B chunk */
				const uint32_t pk = p0 + q / 4u;

				if (pk < npkt) {
					const d_u32x4 v = dld<NT>(src + (size_t)p0 * 4u + q);

					x = v.x ^ v.y ^ v.z ^ v.w;
				} else {
					x = 0u;
				}
				x ^= __shfl_xor(x, 1, 64);
				x ^= __shfl_xor(x, 2, 64);
				if ((q & 3u) == 0u && pk < npkt)
					out[pk] = x;
			}
		} else if (PAT == 1) {
			const uint32_t pk = p0 + tid;

			if (pk < npkt) {
#pragma unroll
				for (int k = 0; k < 4; ++k) {
					const d_u32x4 v = dld<NT>(src + (size_t)pk * 4u + k);

					x ^= v.x ^ v.y ^ v.z ^ v.w;
				}
				out[pk] = x;
			}
		} else {
#pragma unroll
			for (int k = 0; k < 4; ++k) {
				const uint32_t q = k * DBLOCK + tid;
				const uint32_t pk = p0 + q / 4u;
				d_u32x4 v = {0u, 0u, 0u, 0u};

				if (pk < npkt)
					v = dld<NT>(src + (size_t)p0 * 4u + q);
				uint32_t *r = lds + (q / 4u) * 17u + (q & 3u) * 4u;

				r[0] = v.x;
				r[1] = v.y;
				r[2] = v.z;
				r[3] = v.w;
			}
			__syncthreads();
			const uint32_t pk = p0 + tid;
#pragma unroll
			for (int k = 0; k < 16; ++k)
				x ^= lds[tid * 17u + k];
			if (pk < npkt)
				out[pk] = x;
			__syncthreads();
		}
	}
}

template <int PAT, bool NT>
static hipError_t diag_launch(const void *src, uint32_t npkt, uint32_t *out, uint32_t grid,
			      hipStream_t s)
{
	hipLaunchKernelGGL((odpg_diag_stream_kernel<PAT, NT>), dim3(grid), dim3(DBLOCK), 0, s,
			   (const d_u32x4 *)src, npkt, out);
	return hipGetLastError();
}

extern "C" int odpg_diag_stream(odpg_ctx_t *ctx, const void *src, uint32_t npkt, uint32_t *out,
				int pattern, uint32_t grid)
{
	if (!ctx || !src || !out)
		return -EINVAL;
	if (npkt == 0)
		return 0;
	hipStream_t s = (hipStream_t)odpg_ctx_stream(ctx);
	const uint32_t ntiles = (npkt + DBLOCK - 1) / DBLOCK;

	if (grid == 0 || grid > ntiles)
		grid = ntiles;
	hipError_t e;

	switch (pattern) {
	case 0x00: e = diag_launch<0, false>(src, npkt, out, grid, s); break;
	case 0x01: e = diag_launch<1, false>(src, npkt, out, grid, s); break;
	case 0x02: e = diag_launch<2, false>(src, npkt, out, grid, s); break;
	case 0x10: e = diag_launch<0, true>(src, npkt, out, grid, s); break;
	case 0x11: e = diag_launch<1, true>(src, npkt, out, grid, s); break;
	case 0x12: e = diag_launch<2, true>(src, npkt, out, grid, s); break;
	default: return -EINVAL;
	}
	return e == hipSuccess ? 0 : -EIO;
}
