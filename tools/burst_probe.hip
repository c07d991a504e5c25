/*
 * burst_probe.hip -- does the length of each lane's contiguous PCM burst
 * set K1's write rate?  The store half of K1 on C3's shape, nothing else:
 * 125,000 chunks of 40 eblocks (5,120 B of PCM each, one per lane, 1,954
 * waves in 489 four-wave workgroups), every lane writing its chunk front to
 * back, non-temporal, 16 B per lane per instruction.  B = the bytes a lane
 * writes contiguously before the wave moves on:
 *   B = 128: K1's pattern (8 lanes cover one lane's 128-B line: eight whole
 *            lines of eight chunks per instruction)
 *   B = 256, 512: 16, 32 lanes cover one chunk's B bytes
 *   B = 0:   the same bytes as one contiguous stream (lane-linear)
 * Optionally a read stream beside it (R = 1: each lane also reads its
 * chunk's share of a 330 MB input, 264 B per 512 B written, as K1's DMA
 * does, through plain 16-B loads summed into a dummy store).
 * Prints one JSON line per case: median ms of 15 launches, write TB/s.
 *
 * build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -o /tmp/burst_probe tools/burst_probe.hip
 */
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <vector>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
	fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); exit(1); } } while (0)

#define NCH 125000u
#define CB 5120u		/* PCM bytes per chunk */
#define XB 2640u		/* XA bytes per chunk */

template <int B, bool RD>
__global__ __launch_bounds__(256, 2) void
k_burst(uint8_t *out, const uint8_t *in, uint32_t *sink)
{
	const uint32_t w = blockIdx.x * 4 + threadIdx.x / 64, lane = threadIdx.x & 63;
	const uint32_t c0 = w * 64;
	u32x4 acc = { lane, w, 0u, 0x5a5a5a5au };
	/* per outer step every lane of the wave has written 512 B of its
	 * chunk (4 eblocks: one K1 super-step) */
	for (uint32_t s = 0; s < CB / 512; s++) {
		if constexpr (RD) {
			/* 264 B of the lane's own XA run, 16 B at a time (K1's DMA
			 * reads 17 pieces per lane per super-step) */
			const uint32_t q = c0 + lane;
			if (q < NCH) {
#pragma unroll
				for (int k = 0; k < 16; k++)
					acc += *(const u32x4 *)(in + (uint64_t)q * XB + s * 264u +
					    16u * k);
			}
		}
		if constexpr (B == 0) {
			/* the wave's 64 chunks as one contiguous span: instruction i
			 * covers bytes [1024 i, 1024 i + 1024) of the span's s-th
			 * 32 KiB */
			uint8_t *span = out + (uint64_t)c0 * CB + (uint64_t)s * 64u * 512u;
			for (int i = 0; i < 32; i++) {
				const uint64_t off = (uint64_t)i * 1024u + lane * 16u;
				if ((uint64_t)c0 * CB + (uint64_t)s * 32768u + off + 16u <=
				    (uint64_t)NCH * CB)
					__builtin_nontemporal_store(acc, (u32x4 *)(span + off));
			}
		} else {
			static_assert(B == 128 || B == 256 || B == 512, "burst");
			constexpr int LPC = B / 16;		/* lanes per chunk burst */
			constexpr int CPI = 64 / LPC;		/* chunks per instruction */
			/* 64 chunks x 512 B = 32 instructions; each writes B bytes
			 * of CPI chunks; 512 / B rounds per chunk group */
			for (int g = 0; g < 64 / CPI; g++) {
				for (int r = 0; r < 512 / B; r++) {
					const uint32_t q = c0 + g * CPI + lane / LPC;
					const uint64_t off = (uint64_t)q * CB + s * 512u + r * B +
					    (lane % LPC) * 16u;
					if (q < NCH)
						__builtin_nontemporal_store(acc, (u32x4 *)(out + off));
				}
			}
		}
	}
	if (acc.x == 0xdeadbeefu)
		sink[0] = acc.y;
}

template <int B, bool RD>
static void
run(uint8_t *out, const uint8_t *in, uint32_t *sink, const char *name)
{
	const uint32_t waves = (NCH + 63) / 64, grid = (waves + 3) / 4;
	hipEvent_t a, b;
	CHECK(hipEventCreate(&a));
	CHECK(hipEventCreate(&b));
	std::vector<float> ms;
	for (int it = 0; it < 18; it++) {
		CHECK(hipEventRecord(a, 0));
		hipLaunchKernelGGL((k_burst<B, RD>), dim3(grid), dim3(256), 0, 0, out, in, sink);
		CHECK(hipEventRecord(b, 0));
		CHECK(hipEventSynchronize(b));
		float t;
		CHECK(hipEventElapsedTime(&t, a, b));
		if (it >= 3)
			ms.push_back(t);
	}
	std::sort(ms.begin(), ms.end());
	const double med = ms[ms.size() / 2];
	const double wb = (double)NCH * CB, rb = RD ? (double)NCH * 264.0 * (CB / 512) : 0.0;
	printf("{\"case\": \"%s\", \"burst_B\": %d, \"read\": %d, \"ms\": %.4f, "
	    "\"write_TBps\": %.3f, \"total_TBps\": %.3f}\n", name, B, (int)RD, med,
	    wb / med / 1e9, (wb + rb) / med / 1e9);
	fflush(stdout);
	CHECK(hipEventDestroy(a));
	CHECK(hipEventDestroy(b));
}

int
main()
{
	uint8_t *out, *in;
	uint32_t *sink;
	CHECK(hipMalloc(&out, (size_t)NCH * CB));
	CHECK(hipMalloc(&in, (size_t)NCH * XB + 4096));
	CHECK(hipMalloc(&sink, 64));
	CHECK(hipMemset(in, 1, (size_t)NCH * XB + 4096));
	for (int rep = 0; rep < 2; rep++) {
		run<128, false>(out, in, sink, "k1_lines");
		run<256, false>(out, in, sink, "burst256");
		run<512, false>(out, in, sink, "burst512");
		run<0, false>(out, in, sink, "contiguous");
		run<128, true>(out, in, sink, "k1_lines+read");
		run<256, true>(out, in, sink, "burst256+read");
		run<512, true>(out, in, sink, "burst512+read");
		run<0, true>(out, in, sink, "contiguous+read");
	}
	CHECK(hipDeviceSynchronize());
	return 0;
}
