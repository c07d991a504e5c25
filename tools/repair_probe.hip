/*
 * repair_probe.hip -- cost per block of K2's one-lane repair (fix_chunk),
 * isolated: every active lane re-decodes one chunk of C eblocks of a random
 * 8-bit stereo stream from a random state against random "old" PCM, so no
 * repair ever meets the stored trajectory and each runs its whole chunk.
 * The slope over C is the per-block cost; active lanes per wave and waves
 * per workgroup show whether lanes of a wave (their scattered windows and
 * stores) or waves of a CU slow each other down.
 *
 * build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -Ibjxa_amd/csrc -Iinclude \
 *            -o dbg/repair_probe tools/repair_probe.hip
 */
#include "xa_decode.hip"
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
	fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); exit(1); } } while (0)

template <bool BUF>
__global__ __launch_bounds__(256) void
k_rep(xa_dec_args a, uint32_t lanes_per_wave, uint32_t *sink)
{
	const uint32_t lane = threadIdx.x & 63, w = blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64;
	if (lane >= lanes_per_wave)
		return;
	const uint32_t q = 1 + w * 64 + lane;
	uint2 ex;
	const bool met = fix_chunk<8, 2, BUF>(a, q,
	    make_uint2(0x12345678u ^ q, 0x0badf00du + q), ex);
	if (met)
		atomicAdd(sink, 1u);
}

int
main()
{
	const uint32_t nchunks = 64 * 1024 + 2, Cmax = 64;
	const uint64_t eb = (uint64_t)nchunks * Cmax;
	uint8_t *src, *dst, *pristine;
	uint2 *ge;
	uint32_t *sink;
	CHECK(hipMalloc(&src, eb * 66));
	CHECK(hipMalloc(&dst, eb * 128));
	CHECK(hipMalloc(&pristine, eb * 128));
	CHECK(hipMalloc(&ge, 2 * nchunks * sizeof(uint2)));
	CHECK(hipMalloc(&sink, 4));
	{
		uint8_t *h = (uint8_t *)malloc(eb * 128);
		uint64_t s = 88172645463325252ull;
		for (uint64_t i = 0; i < eb * 128; i += 8) {
			s ^= s << 13; s ^= s >> 7; s ^= s << 17;
			memcpy(h + i, &s, 8);
		}
		/* profiles: gain 4, range 12 (mix W) */
		for (uint64_t i = 0; i < eb * 2; i++)
			h[i * 33] = 0x4c;
		CHECK(hipMemcpy(src, h, eb * 66, hipMemcpyHostToDevice));
		CHECK(hipMemcpy(pristine, h + 7, eb * 128 - 64, hipMemcpyHostToDevice));
		free(h);
	}
	CHECK(hipMemset(sink, 0, 4));
	hipEvent_t e0, e1;
	CHECK(hipEventCreate(&e0));
	CHECK(hipEventCreate(&e1));
	struct { uint32_t C, lanes, wpb, grid; } cases[] = {
		{16, 1, 1, 1}, {64, 1, 1, 1},
		{16, 64, 1, 1}, {64, 64, 1, 1},
		{16, 64, 4, 1}, {64, 64, 4, 1},
		{16, 64, 4, 256}, {64, 64, 4, 256},
		{16, 16, 4, 256}, {64, 16, 4, 256},
	};
	for (int rep = 0; rep < 2; rep++)
	for (auto &c : cases) {
		xa_dec_args a = {};
		a.src = src;
		a.dst = dst;
		a.eblocks = (uint32_t)((uint64_t)nchunks * c.C);
		a.pcm_bytes = (uint64_t)a.eblocks * 128;
		a.nchunks = nchunks;
		a.C = c.C;
		a.W = 8;
		a.g = ge;
		a.e = ge + nchunks;
		for (int b = 0; b < 2; b++) {
			/* each launch starts from the pristine "old" PCM (a repair
			 * rewrites it, and a later launch would then meet it) */
			float sum = 0.0f;
			for (int i = 0; i < 6; i++) {
				CHECK(hipMemcpyAsync(dst, pristine, eb * 128, hipMemcpyDeviceToDevice, 0));
				CHECK(hipEventRecord(e0, 0));
				if (b)
					hipLaunchKernelGGL(k_rep<true>, dim3(c.grid), dim3(64 * c.wpb), 0, 0, a, c.lanes, sink);
				else
					hipLaunchKernelGGL(k_rep<false>, dim3(c.grid), dim3(64 * c.wpb), 0, 0, a, c.lanes, sink);
				CHECK(hipEventRecord(e1, 0));
				CHECK(hipEventSynchronize(e1));
				float ms;
				CHECK(hipEventElapsedTime(&ms, e0, e1));
				if (i)
					sum += ms;
			}
			float ms[2] = {0.0f, sum / 5};
			printf("{\"C\": %u, \"lanes_per_wave\": %u, \"waves_per_wg\": %u, \"grid\": %u, \"buf\": %d, \"us\": %.2f}\n",
			    c.C, c.lanes, c.wpb, c.grid, b, ms[1] * 1000.0f);
		}
	}
	uint32_t hs;
	CHECK(hipMemcpy(&hs, sink, 4, hipMemcpyDeviceToHost));
	printf("{\"met\": %u}\n", hs);
	return 0;
}
