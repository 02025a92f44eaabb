/* SPDX-License-Identifier: BSD-3-Clause
 *
 * Commit of the loopback_recv pktio counters (in_packets, in_octets,
 * in_errors, in_discards; pktio/loop.c:304-374) from per-wave sums into the
 * caller's 64-bit counters.
 *
 * Measured on MI355X (C2 launch, ~6000 resident waves, 17.3 us without
 * counters), in-kernel grid reductions all cost more than the work they
 * count:
 *  - one device-scope atomic per workgroup on the caller's four words:
 *    +30 us (the workgroups finish within a microsecond and serialise on
 *    one address each);
 *  - acquire/release tickets: +27 us (an agent-scope release writes back
 *    the XCD's L2, once per workgroup);
 *  - spread slots + relaxed group and grid tickets: +4.3 us (four dependent
 *    atomic round trips on the last wave);
 *  - packed ticket|sum words, one returning atomic per word per wave:
 *    +9.4 us (returning atomics serialise per cache line).
 * Non-returning adds into SRED_GROUPS spread slots (one 64 B line each) cost
 * +0.4 us. So waves only add (no return) into the context's slots, and a
 * one-wave fold kernel queued behind the classify launch on the same stream
 * moves the slot sums into the caller's counters and re-zeroes the slots.
 */
#ifndef ODPG_STATS_COMMIT_H
#define ODPG_STATS_COMMIT_H

#include <hip/hip_runtime.h>
#include <stdint.h>

#define SRED_GROUPS 64u
#define SRED_BYTES (SRED_GROUPS * 64u)   /* u64[64][8], words 0..3 used */

#define SC_RELAXED(op, ...) __hip_atomic_##op(__VA_ARGS__, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)

/* Called by every wave of the grid, once, with wave-uniform sums v[0..3]. */
__device__ __forceinline__ void stats_commit_wave(const uint64_t (&v)[4], uint64_t *sred)
{
	const uint32_t gw = blockIdx.x * (blockDim.x / 64u) + threadIdx.x / 64u;

	if (__lane_id() == 0u) {
		uint64_t *slot = sred + (gw % SRED_GROUPS) * 8u;

#pragma unroll
		for (int w = 0; w < 4; ++w)
			if (v[w])
				SC_RELAXED(fetch_add, slot + w, v[w]);
	}
}

#endif
