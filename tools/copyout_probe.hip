/*
 * copyout_probe.hip -- the duplex route's copy-out (HBM -> pinned host
 * memory, xa_gpu.hip xa_slab_out) runs 43-44 GB/s per 16 MiB slab against
 * 55 GB/s for one long kernel write (R6-7).  Which part costs it?
 *
 * On CDNA one counter (vmcnt) covers loads and stores, so a wave that loads
 * after storing waits for its stores' PCIe round trip.  Cases, 256 MiB in
 * all, medians of 5 runs:
 *   slab_out      the shipped kernel, 16 launches of 16 MiB (128 workgroups)
 *   slab_out_one  the same kernel, one launch of 256 MiB
 *   split         loader and storer waves: two waves of each workgroup load
 *                 HBM into an LDS ring, the other two store from it to the
 *                 host and never load global memory, so nothing waits on a
 *                 store; 16 launches of 16 MiB
 *   split_one     the same, one launch
 *   store_only    constant stores, 16 launches (no loads at all)
 *
 * build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -o tools/bin/copyout_probe \
 *            tools/copyout_probe.hip
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
#define U	8

/* the shipped copy-out's loop */
__global__ __launch_bounds__(256) void
k_slab_out(const uint4 *src, uint4 *dst, uint64_t n16)
{
	const uint64_t step = (uint64_t)gridDim.x * 256u * U;
	uint64_t i = blockIdx.x * 256ull * U + threadIdx.x;
	for (; i + 256u * (U - 1) < n16; i += step) {
		uint4 v[U];
#pragma unroll
		for (int u = 0; u < U; u++)
			v[u] = src[i + 256u * u];
#pragma unroll
		for (int u = 0; u < U; u++)
			dst[i + 256u * u] = v[u];
	}
	for (int u = 0; u < U; u++)
		if (i + 256u * u < n16)
			dst[i + 256u * u] = src[i + 256u * u];
}

/*
 * Loader / storer split.  Workgroup of 256 = 4 waves; wave p (0, 1) loads
 * for wave p + 2.  Per pair an LDS ring of R stages of 64 lanes x SU x 16 B;
 * flag[stage] = 2k + 1 once round k's data is in, 2k + 2 once it is out.
 * Every spin is bounded (a wave that gives up leaves garbage, never a hang).
 */
#define SU	4
#define R	8
#define SPIN	(1u << 22)

__global__ __launch_bounds__(256) void
k_split(const uint4 *src, uint4 *dst, uint64_t n16)
{
	__shared__ uint4 ring[2][R][SU * 64];
	__shared__ uint32_t flag[2][R];
	const uint32_t wave = threadIdx.x >> 6, lane = threadIdx.x & 63u;
	const uint32_t pair = wave & 1u;
	if (threadIdx.x < 2 * R)
		flag[threadIdx.x / R][threadIdx.x % R] = 0u;
	__syncthreads();
	/* pieces of SU*64 uint4 per (pair, round), pairs interleaved over the grid */
	const uint64_t per = (uint64_t)SU * 64u;
	const uint64_t npieces = (n16 + per - 1) / per;
	const uint64_t first = (uint64_t)blockIdx.x * 2u + pair;
	const uint64_t stride = (uint64_t)gridDim.x * 2u;
	uint32_t k = 0;
	if (wave < 2) {
		for (uint64_t p = first; p < npieces; p += stride, k++) {
			const uint32_t s = k % R, want = 2u * (k / R);
			uint4 v[SU];
#pragma unroll
			for (int u = 0; u < SU; u++) {
				const uint64_t j = p * per + (uint64_t)u * 64u + lane;
				v[u] = j < n16 ? src[j] : make_uint4(0, 0, 0, 0);
			}
			for (uint32_t t = 0; t < SPIN && __hip_atomic_load(&flag[pair][s],
			    __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) != want; t++)
				__builtin_amdgcn_s_sleep(1);
#pragma unroll
			for (int u = 0; u < SU; u++)
				ring[pair][s][u * 64 + lane] = v[u];
			if (lane == 0)
				__hip_atomic_store(&flag[pair][s], want + 1u, __ATOMIC_RELEASE,
				    __HIP_MEMORY_SCOPE_WORKGROUP);
		}
	} else {
		for (uint64_t p = first; p < npieces; p += stride, k++) {
			const uint32_t s = k % R, want = 2u * (k / R) + 1u;
			for (uint32_t t = 0; t < SPIN && __hip_atomic_load(&flag[pair][s],
			    __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) != want; t++)
				__builtin_amdgcn_s_sleep(1);
			uint4 v[SU];
#pragma unroll
			for (int u = 0; u < SU; u++)
				v[u] = ring[pair][s][u * 64 + lane];
			if (lane == 0)
				__hip_atomic_store(&flag[pair][s], want + 1u, __ATOMIC_RELEASE,
				    __HIP_MEMORY_SCOPE_WORKGROUP);
#pragma unroll
			for (int u = 0; u < SU; u++) {
				const uint64_t j = p * per + (uint64_t)u * 64u + lane;
				if (j < n16)
					dst[j] = v[u];
			}
		}
	}
}

__global__ __launch_bounds__(256) void
k_store_only(uint4 *dst, uint64_t n16)
{
	const uint4 v = make_uint4(threadIdx.x, blockIdx.x, 1u, 2u);
	for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n16;
	    i += (uint64_t)gridDim.x * 256u)
		dst[i] = v;
}

int
main(int argc, char **argv)
{
	const int grid = argc > 1 ? atoi(argv[1]) : 128;
	uint8_t *d_src, *h_dst, *d_dst;
	CHECK(hipMalloc(&d_src, NSLAB * SLAB));
	CHECK(hipMemset(d_src, 0x5a, NSLAB * SLAB));
	CHECK(hipHostMalloc((void **)&h_dst, NSLAB * SLAB, hipHostMallocDefault));
	CHECK(hipHostGetDevicePointer((void **)&d_dst, h_dst, 0));
	hipStream_t s;
	CHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
	hipEvent_t a, b;
	CHECK(hipEventCreate(&a));
	CHECK(hipEventCreate(&b));
	const char *names[] = { "slab_out", "slab_out_one", "split", "split_one",
	    "store_only" };
	for (int rep = 0; rep < 2; rep++)
	for (int c = 0; c < 5; c++) {
		std::vector<float> ms;
		for (int it = 0; it < 6; it++) {
			memset(h_dst, 0, 4096);
			CHECK(hipEventRecord(a, s));
			const bool one = c == 1 || c == 3;
			const int launches = one ? 1 : NSLAB;
			const size_t len = one ? NSLAB * SLAB : SLAB;
			for (int k = 0; k < launches; k++) {
				const uint4 *sp = (const uint4 *)(d_src + k * len);
				uint4 *dp = (uint4 *)(d_dst + k * len);
				if (c <= 1)
					hipLaunchKernelGGL(k_slab_out, dim3(grid), dim3(256), 0, s,
					    sp, dp, (uint64_t)(len / 16));
				else if (c <= 3)
					hipLaunchKernelGGL(k_split, dim3(grid), dim3(256), 0, s,
					    sp, dp, (uint64_t)(len / 16));
				else
					hipLaunchKernelGGL(k_store_only, dim3(grid), dim3(256), 0, s,
					    dp, (uint64_t)(len / 16));
			}
			CHECK(hipGetLastError());
			CHECK(hipEventRecord(b, s));
			CHECK(hipEventSynchronize(b));
			float t;
			CHECK(hipEventElapsedTime(&t, a, b));
			if (it >= 1)
				ms.push_back(t);
		}
		std::sort(ms.begin(), ms.end());
		/* every case but store_only copies the source: check a few words */
		bool ok = true;
		if (c < 4)
			for (size_t o = 0; o < NSLAB * SLAB; o += 1234567)
				ok = ok && h_dst[o] == 0x5a;
		printf("{\"rep\": %d, \"case\": \"%s\", \"grid\": %d, \"ms\": %.3f, "
		    "\"GBps\": %.1f, \"bytes_ok\": %s}\n", rep, names[c], grid,
		    ms[ms.size() / 2], NSLAB * SLAB / ms[ms.size() / 2] / 1e6,
		    ok ? "true" : "false");
		fflush(stdout);
	}
	return 0;
}
