/*
 * store_probe.hip -- is the packed-batch loss a
 * property of writing into one large allocation?  The store half of K1 on
 * C5g's shape, nothing else: 128 PCM images of 8 MiB, each written by 16
 * waves whose 64 lanes own chunks of C eblocks (128 B per eblock, so the
 * lane stride is C * 128 B), one 128-B line per lane per step, stored as K1
 * stores them (lane l writes piece l % 8 of lines l / 8 + 8 i, i < 8: eight
 * whole lines per instruction, non-temporal).  The images are either 128
 * hipMallocs of their own or back to back in one hipMalloc.  Prints one
 * JSON line per case: median ms of 15 launches and write TB/s.
 *
 * build: hipcc --offload-arch=gfx950 -O3 -o dbg/store_probe tools/store_probe.hip
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

#define NIMG 128
#define IMG (8u << 20)

/* wave w writes lanes 64 (w % wpi) .. +63 of image w / wpi */
__global__ __launch_bounds__(256, 2) void
k_store(uint8_t *const *img, uint32_t C, uint32_t wpi, uint32_t lanes)
{
	const uint32_t w = blockIdx.x * 4 + threadIdx.x / 64, lane = threadIdx.x & 63;
	const uint32_t im = w / wpi, l0 = (w % wpi) * 64;
	uint8_t *base = img[im];
	const uint64_t cb = (uint64_t)C * 128;
	const u32x4 v = { lane, w, C, 0x5a5a5a5au };
	for (uint32_t s = 0; s < C; s++) {
#pragma unroll
		for (int i = 0; i < 8; i++) {
			const uint32_t j = lane / 8 + 8 * i, q = l0 + j;
			if (q < lanes)
				__builtin_nontemporal_store(v, (u32x4 *)(base + q * cb +
				    (uint64_t)s * 128 + (lane % 8) * 16));
		}
	}
}

static double
run(uint8_t **h_img, uint32_t C)
{
	const uint32_t lanes = IMG / (C * 128), wpi = (lanes + 63) / 64;
	uint8_t **d_img;
	CHECK(hipMalloc(&d_img, NIMG * sizeof(uint8_t *)));
	CHECK(hipMemcpy(d_img, h_img, NIMG * sizeof(uint8_t *), hipMemcpyHostToDevice));
	const uint32_t grid = (NIMG * wpi + 3) / 4;
	hipEvent_t a, b;
	CHECK(hipEventCreate(&a));
	CHECK(hipEventCreate(&b));
	std::vector<float> ms;
	for (int r = 0; r < 18; r++) {
		CHECK(hipEventRecord(a, 0));
		hipLaunchKernelGGL(k_store, dim3(grid), dim3(256), 0, 0, d_img, C, wpi, lanes);
		CHECK(hipEventRecord(b, 0));
		CHECK(hipEventSynchronize(b));
		float t;
		CHECK(hipEventElapsedTime(&t, a, b));
		if (r >= 3)
			ms.push_back(t);
	}
	std::sort(ms.begin(), ms.end());
	CHECK(hipFree(d_img));
	CHECK(hipEventDestroy(a));
	CHECK(hipEventDestroy(b));
	return ms[ms.size() / 2];
}

int
main()
{
	uint8_t *h_sep[NIMG], *h_one[NIMG], *big;
	for (int i = 0; i < NIMG; i++)
		CHECK(hipMalloc(&h_sep[i], IMG));
	CHECK(hipMalloc(&big, (size_t)NIMG * IMG));
	for (int i = 0; i < NIMG; i++)
		h_one[i] = big + (size_t)i * IMG;
	const uint32_t Cs[] = { 64, 68, 40 };
	for (int rep = 0; rep < 2; rep++)
		for (uint32_t C : Cs) {
			for (int k = 0; k < 2; k++) {
				uint8_t **h = k ? h_one : h_sep;
				const uint32_t lanes = IMG / (C * 128);
				const double t = run(h, C);
				const double bytes = (double)NIMG * lanes * C * 128;
				printf("{\"layout\": \"%s\", \"C\": %u, \"rep\": %d, \"ms\": %.4f, "
				    "\"write_TBps\": %.3f}\n", k ? "one" : "separate", C, rep, t,
				    bytes / (t * 1e-3) / 1e12);
			}
		}
	return 0;
}
