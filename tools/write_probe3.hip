/*
 * write_probe3.hip -- does the allocation that holds an output matter to
 * its write rate?  (Round 6: C5g's PCM images decode ~15 % slower packed in
 * one allocation than in one allocation each, whatever their address bits
 * and chunk length, tools/r06v.sh.)
 *
 * One store pattern, K1's: wave w owns 64 rows ("chunks") of 5,120 B (C3's
 * 40 eblocks of stereo PCM); each store instruction writes 8 segments of
 * 128 B (8 lanes x 16 B each) into 8 of the wave's rows, and 8 instructions
 * cover 128 B of all 64 rows.  1,960 waves (C3's grid) = 642 MB per launch.
 * The rows are reached through a pointer table, so the same pattern runs
 * over different allocations:
 *   one      every row in one hipMalloc, back to back
 *   split<m> the same rows in hipMallocs of m MiB each (rows never cross
 *            an allocation; each allocation's rows back to back)
 * Per case: non-temporal stores back to back (K1's), and plain stores after
 * a 1 GiB read that evicts the Infinity Cache.  Median of 10 launches.
 *
 * build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -o tools/bin/write_probe3 \
 *            tools/write_probe3.hip
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

#define ROW	5120u
#define NWAVES	1960u
#define NROWS	(NWAVES * 64u)

template <int NT>
__global__ __launch_bounds__(256) void
kseg(uint8_t *const *rows)
{
	const uint32_t w = blockIdx.x * 4u + (threadIdx.x >> 6);
	const uint32_t lane = threadIdx.x & 63u;
	if (w >= NWAVES)
		return;
	uint8_t *p[8];
#pragma unroll
	for (int j = 0; j < 8; j++)
		p[j] = rows[w * 64u + (uint32_t)j * 8u + lane / 8u] + (lane % 8u) * 16u;
	const u32x4 v = { lane, w, 1u, 2u };
	for (uint32_t o = 0; o < ROW; o += 128u) {
#pragma unroll
		for (int j = 0; j < 8; j++) {
			if (NT)
				__builtin_nontemporal_store(v, (u32x4 *)(p[j] + o));
			else
				*(u32x4 *)(p[j] + o) = v;
		}
	}
}

__global__ __launch_bounds__(256) void
kflush(const u32x4 *in, uint64_t n, uint32_t *sink)
{
	u32x4 acc = { 0u, 0u, 0u, 0u };
	for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += gridDim.x * 256ull)
		acc ^= in[i];
	if ((acc.x ^ acc.y ^ acc.z ^ acc.w) == 0x9e3779b9u)
		sink[0] = 1u;	/* practically never: keeps the loads */
}

#define FLUSH_BYTES (1ull << 30)
static u32x4 *g_fl;
static uint32_t *g_sink;

static float
time_case(uint8_t **d_rows, bool nt, bool flush)
{
	hipEvent_t a, b;
	CHECK(hipEventCreate(&a));
	CHECK(hipEventCreate(&b));
	std::vector<float> ms;
	for (int it = 0; it < 13; it++) {
		if (flush)
			hipLaunchKernelGGL(kflush, dim3(2048), dim3(256), 0, 0, g_fl,
			    FLUSH_BYTES / 16, g_sink);
		CHECK(hipEventRecord(a, 0));
		if (nt)
			hipLaunchKernelGGL(kseg<1>, dim3(NWAVES / 4), dim3(256), 0, 0, d_rows);
		else
			hipLaunchKernelGGL(kseg<0>, dim3(NWAVES / 4), dim3(256), 0, 0, d_rows);
		CHECK(hipEventRecord(b, 0));
		CHECK(hipEventSynchronize(b));
		float t;
		CHECK(hipEventElapsedTime(&t, a, b));
		if (it >= 3)
			ms.push_back(t);
	}
	std::sort(ms.begin(), ms.end());
	CHECK(hipEventDestroy(a));
	CHECK(hipEventDestroy(b));
	return ms[ms.size() / 2];
}

/* rows in allocations of `mib` MiB (0: one allocation for all) */
static void
run(unsigned mib, int rep)
{
	const uint64_t total = (uint64_t)NROWS * ROW;
	const uint64_t per = mib ? ((uint64_t)mib << 20) / ROW : NROWS;
	std::vector<void *> allocs;
	std::vector<uint8_t *> rows(NROWS);
	for (uint64_t r = 0; r < NROWS; r += per) {
		const uint64_t k = std::min<uint64_t>(per, NROWS - r);
		void *p;
		CHECK(hipMalloc(&p, k * ROW));
		CHECK(hipMemset(p, 0, k * ROW));
		allocs.push_back(p);
		for (uint64_t i = 0; i < k; i++)
			rows[r + i] = (uint8_t *)p + i * ROW;
	}
	uint8_t **d_rows;
	CHECK(hipMalloc(&d_rows, NROWS * sizeof(uint8_t *)));
	CHECK(hipMemcpy(d_rows, rows.data(), NROWS * sizeof(uint8_t *),
	    hipMemcpyHostToDevice));
	const float t_nt = time_case(d_rows, true, false);
	const float t_pl = time_case(d_rows, false, true);
	printf("{\"rep\": %d, \"case\": \"%s%u\", \"allocations\": %zu, \"MB\": %.1f, "
	    "\"nt_back_to_back_ms\": %.4f, \"nt_TBps\": %.3f, "
	    "\"plain_after_flush_ms\": %.4f, \"plain_TBps\": %.3f}\n", rep,
	    mib ? "split" : "one", mib, allocs.size(), total / 1e6, t_nt,
	    total / t_nt / 1e9, t_pl, total / t_pl / 1e9);
	fflush(stdout);
	CHECK(hipFree(d_rows));
	for (void *p : allocs)
		CHECK(hipFree(p));
}

int
main()
{
	CHECK(hipMalloc(&g_fl, FLUSH_BYTES));
	CHECK(hipMalloc(&g_sink, 64));
	CHECK(hipMemset(g_fl, 1, FLUSH_BYTES));
	const unsigned sizes[] = { 0, 8, 2, 32, 128, 0, 8 };
	for (int rep = 0; rep < 2; rep++)
		for (unsigned m : sizes)
			run(m, rep);
	return 0;
}
