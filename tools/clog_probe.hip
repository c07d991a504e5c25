/*
 * clog_probe.hip -- does a kernel storing into pinned host memory (PCIe
 * bound) slow other kernels that write HBM at the same time?  In the duplex
 * route's trace a slab decode that ran beside the copy-out kernel took
 * 0.36 ms instead of 0.05 (R6-7).
 *
 * s_out: 16 back-to-back copy-outs of 16 MiB HBM -> pinned host (~5 ms).
 * s_w:   a chain of 40 HBM -> HBM copies of 16 MiB (the "decode" stand-in),
 *        started together with the copy-outs; its time is reported.
 * Each with the two streams' CU masks taken several ways:
 *   alone        the HBM chain with no copy-out running
 *   every4       copy-out on CUs c % 4 == 0 (64), chain on the rest (the route)
 *   first64      copy-out on CUs 0-63, chain on 64-255
 *   every8x2     copy-out on c % 8 in {0, 1} (64), chain on the rest
 *   nomask       both streams unmasked
 * Median of 5.
 *
 * build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -o tools/bin/clog_probe \
 *            tools/clog_probe.hip
 */
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <algorithm>
#include <vector>

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
	fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); exit(1); } } while (0)

#define SLAB	((size_t)16 << 20)
#define NSLAB	16
#define NW	40

__global__ __launch_bounds__(256) void
k_copy(const uint4 *src, uint4 *dst, uint64_t n16)
{
	for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n16;
	    i += (uint64_t)gridDim.x * 256u)
		dst[i] = src[i];
}

int
main()
{
	int ncu = 0;
	CHECK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
	uint8_t *src, *a, *b, *h, *d_h;
	CHECK(hipMalloc(&src, NSLAB * SLAB));
	CHECK(hipMalloc(&a, SLAB));
	CHECK(hipMalloc(&b, SLAB));
	CHECK(hipMemset(src, 1, NSLAB * SLAB));
	CHECK(hipMemset(a, 2, SLAB));
	CHECK(hipHostMalloc((void **)&h, NSLAB * SLAB, hipHostMallocDefault));
	CHECK(hipHostGetDevicePointer((void **)&d_h, h, 0));
	const char *names[] = { "alone", "every4", "first64", "every8x2", "nomask" };
	hipEvent_t w0, w1;
	CHECK(hipEventCreate(&w0));
	CHECK(hipEventCreate(&w1));
	for (int rep = 0; rep < 2; rep++)
	for (int m = 0; m < 5; m++) {
		uint32_t mo[64] = { 0 }, mw[64] = { 0 };
		for (int c = 0; c < ncu; c++) {
			bool out = m == 1 ? c % 4 == 0 : m == 2 ? c < 64 :
			    m == 3 ? (c % 8 == 0 || c % 8 == 1) : false;
			(out ? mo : mw)[c / 32] |= 1u << (c % 32);
		}
		hipStream_t s_out, s_w;
		if (m == 0 || m == 4) {
			CHECK(hipStreamCreateWithFlags(&s_out, hipStreamNonBlocking));
			CHECK(hipStreamCreateWithFlags(&s_w, hipStreamNonBlocking));
		} else {
			CHECK(hipExtStreamCreateWithCUMask(&s_out, (uint32_t)(ncu + 31) / 32, mo));
			CHECK(hipExtStreamCreateWithCUMask(&s_w, (uint32_t)(ncu + 31) / 32, mw));
		}
		std::vector<float> ms;
		for (int it = 0; it < 6; it++) {
			CHECK(hipDeviceSynchronize());
			if (m != 0)
				for (int k = 0; k < NSLAB; k++)
					hipLaunchKernelGGL(k_copy, dim3(128), dim3(256), 0, s_out,
					    (const uint4 *)(src + k * SLAB), (uint4 *)(d_h + k * SLAB),
					    (uint64_t)(SLAB / 16));
			CHECK(hipEventRecord(w0, s_w));
			for (int j = 0; j < NW; j++)
				hipLaunchKernelGGL(k_copy, dim3(512), dim3(256), 0, s_w,
				    (const uint4 *)a, (uint4 *)b, (uint64_t)(SLAB / 16));
			CHECK(hipEventRecord(w1, s_w));
			CHECK(hipEventSynchronize(w1));
			float t;
			CHECK(hipEventElapsedTime(&t, w0, w1));
			CHECK(hipDeviceSynchronize());
			if (it >= 1)
				ms.push_back(t);
		}
		std::sort(ms.begin(), ms.end());
		printf("{\"rep\": %d, \"masks\": \"%s\", \"hbm_chain_ms\": %.3f, "
		    "\"per_copy_us\": %.1f}\n", rep, names[m], ms[ms.size() / 2],
		    1000.0 * ms[ms.size() / 2] / NW);
		fflush(stdout);
		CHECK(hipStreamDestroy(s_out));
		CHECK(hipStreamDestroy(s_w));
	}
	return 0;
}
