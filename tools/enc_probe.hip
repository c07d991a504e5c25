/*
 * enc_probe.hip -- the memory floor of the encode kernel's pattern
 * (xa_encode.hip xa_encode_waves<8,2> on C3-shaped PCM: 5,000,000 stereo
 * eblocks = 640 MB of PCM in, 330 MB of XA out): the same grid (one wave
 * per 64 four-block groups, four waves per workgroup, 64 KiB of LDS per
 * workgroup), the same 16-B LDS-DMA of the wave's 16 KiB of PCM and the
 * same non-temporal 16-B stores of its 8,448 B of XA, and nothing in
 * between (the XA written is the first 8,448 B of the staged PCM).
 * Prints one JSON line per pass: median ms of 15 launches.
 * 
 *
 * build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -o /tmp/enc_probe tools/enc_probe.hip
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
#define LDS_PTR(p) ((__attribute__((address_space(3))) void *)(p))

#define EBLOCKS 5000000ull
#define NGROUPS (EBLOCKS / 2)		/* stereo: two eblocks per group */
#define NOUT (64 * 33 * 4)		/* XA bytes per wave */

__global__ __launch_bounds__(256) void
k_enc(const uint8_t *src, uint8_t *dst)
{
	__shared__ __attribute__((aligned(16))) uint8_t lds[4 * 16384];
	const int lane = threadIdx.x & 63;
	const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
	uint8_t *buf = lds + wv * 16384;
	const uint64_t w = (uint64_t)blockIdx.x * 4 + wv;
	if (w * 64 >= NGROUPS)
		return;
	const uint64_t base = w * 16384u;
#pragma unroll
	for (int i = 0; i < 16; i++)
		__builtin_amdgcn_global_load_lds(src + base + i * 1024 + lane * 16,
		    LDS_PTR(buf + i * 1024), 16, 0, 0);
	asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
	__builtin_amdgcn_wave_barrier();
	uint8_t *d = dst + w * NOUT;
	for (int i = 0; i < (NOUT / 16 + 63) / 64; i++) {
		const int k = 64 * i + lane;
		if (k < NOUT / 16)
			__builtin_nontemporal_store(*(const u32x4 *)(buf + 16 * k),
			    (u32x4 *)(d + 16 * k));
	}
}

int
main()
{
	uint8_t *src, *dst;
	const uint64_t nw = (NGROUPS + 63) / 64;
	CHECK(hipMalloc(&src, nw * 16384));
	CHECK(hipMalloc(&dst, nw * NOUT));
	CHECK(hipMemset(src, 3, nw * 16384));
	const unsigned grid = (unsigned)((nw + 3) / 4);
	hipEvent_t a, b;
	CHECK(hipEventCreate(&a));
	CHECK(hipEventCreate(&b));
	for (int rep = 0; rep < 2; rep++) {
		std::vector<float> ms;
		for (int it = 0; it < 18; it++) {
			CHECK(hipEventRecord(a, 0));
			hipLaunchKernelGGL(k_enc, dim3(grid), dim3(256), 0, 0, src, dst);
			CHECK(hipEventRecord(b, 0));
			CHECK(hipEventSynchronize(b));
			float t;
			CHECK(hipEventElapsedTime(&t, a, b));
			if (it >= 3)
				ms.push_back(t);
		}
		std::sort(ms.begin(), ms.end());
		const double med = ms[ms.size() / 2];
		printf("{\"case\": \"encode_pattern\", \"ms\": %.4f, \"alg_TBps\": %.3f}\n", med,
		    (double)EBLOCKS * 194.0 / med / 1e9);
		fflush(stdout);
	}
	return 0;
}
