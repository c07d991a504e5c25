/*
 * write_probe.hip -- the chip's write ceiling: 640 MiB written by a
 * grid-stride kernel of 256-thread workgroups, 16 B per lane per store,
 * plain or non-temporal, at 256 .. 4096 workgroups (1 .. 16 per CU).
 * Prints one JSON line per case: median ms of 10 launches, write TB/s.
 * (profiles/r05_write_probe.json)
 *
 * build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -o /tmp/wprobe tools/write_probe.hip
 */
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <algorithm>
#include <vector>
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); exit(1); } } while (0)
#define BYTES (640ull << 20)
/* grid-stride write of BYTES, 16 B per lane per store; POL 0 plain, 1 nt */
template <int POL>
__global__ __launch_bounds__(256) void kw(uint8_t *out, uint64_t per_wg)
{
	const u32x4 v = { threadIdx.x, blockIdx.x, 1u, 2u };
	uint8_t *p = out + (uint64_t)blockIdx.x * per_wg;
	for (uint64_t o = threadIdx.x * 16u; o < per_wg; o += 4096u) {
		if (POL) __builtin_nontemporal_store(v, (u32x4 *)(p + o));
		else *(u32x4 *)(p + o) = v;
	}
}
template <int POL> static void run(uint8_t *out, int wgs)
{
	const uint64_t per = BYTES / wgs / 4096 * 4096;
	hipEvent_t a, b; CHECK(hipEventCreate(&a)); CHECK(hipEventCreate(&b));
	std::vector<float> ms;
	for (int it = 0; it < 13; it++) {
		CHECK(hipEventRecord(a, 0));
		hipLaunchKernelGGL(kw<POL>, dim3(wgs), dim3(256), 0, 0, out, per);
		CHECK(hipEventRecord(b, 0)); CHECK(hipEventSynchronize(b));
		float t; CHECK(hipEventElapsedTime(&t, a, b)); if (it >= 3) ms.push_back(t);
	}
	std::sort(ms.begin(), ms.end());
	printf("{\"policy\": \"%s\", \"wgs\": %d, \"ms\": %.4f, \"write_TBps\": %.3f}\n", POL ? "nt" : "plain", wgs, ms[5], (double)per * wgs / ms[5] / 1e9);
	fflush(stdout);
}
int main()
{
	uint8_t *out; CHECK(hipMalloc(&out, BYTES));
	for (int rep = 0; rep < 2; rep++)
		for (int wgs : {256, 512, 1024, 2048, 4096}) { run<1>(out, wgs); run<0>(out, wgs); }
	return 0;
}
