/*
 * copyout_probe2.hip -- the duplex route's copy-out streams 16 MiB slabs at
 * 43-44 GB/s inside bjxa_decode (R6-7) but at 55 GB/s alone
 * (tools/copyout_probe.hip).  This rebuilds the route's pipeline around the
 * same copy kernel, one factor at a time: the 4-slot staging ring reused
 * (else a fresh 256 MiB pinned target), the host copying each slot into a
 * pageable buffer before the slot is reused (xa_pool, as the route does),
 * and a 132 MB H2D of registered pageable input on a copy engine at the
 * start.  16 slabs of 16 MiB; host clock from first enqueue to the last
 * slab's host copy; median of 5 runs.
 *
 * build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -pthread \
 *            -o tools/bin/copyout_probe2 tools/copyout_probe2.hip
 */
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <algorithm>
#include <chrono>
#include <vector>

#include "../bjxa_amd/csrc/xa_pool.h"

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
	fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); exit(1); } } while (0)

#define SLAB	((size_t)16 << 20)
#define NSLAB	16
#define SLOTS	4
#define U	8
#define IN_BYTES	((size_t)132 << 20)

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

static double
now_ms(void)
{
	return std::chrono::duration<double, std::milli>(
	    std::chrono::steady_clock::now().time_since_epoch()).count();
}

int
main()
{
	uint8_t *d_src, *d_in, *h_lin, *d_lin, *h_ring, *d_ring;
	CHECK(hipMalloc(&d_src, NSLAB * SLAB));
	CHECK(hipMemset(d_src, 0x5a, NSLAB * SLAB));
	CHECK(hipMalloc(&d_in, IN_BYTES));
	CHECK(hipHostMalloc((void **)&h_lin, NSLAB * SLAB, hipHostMallocDefault));
	CHECK(hipHostGetDevicePointer((void **)&d_lin, h_lin, 0));
	CHECK(hipHostMalloc((void **)&h_ring, SLOTS * SLAB, hipHostMallocDefault));
	CHECK(hipHostGetDevicePointer((void **)&d_ring, h_ring, 0));
	/* pageable input (registered per run, as the route does) and output */
	uint8_t *h_in = (uint8_t *)aligned_alloc(4096, IN_BYTES);
	uint8_t *h_dst = (uint8_t *)aligned_alloc(4096, NSLAB * SLAB);
	memset(h_in, 1, IN_BYTES);
	memset(h_dst, 2, NSLAB * SLAB);
	hipStream_t s_out, s_in;
	CHECK(hipStreamCreateWithFlags(&s_out, hipStreamNonBlocking));
	CHECK(hipStreamCreateWithFlags(&s_in, hipStreamNonBlocking));
	std::vector<hipEvent_t> ev(NSLAB);
	for (hipEvent_t &e : ev)
		CHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
	xa_pool::copy_pool pool(xa_pool::pool_threads());

	/* CU-masked copy-out streams, as the route makes them (xa_gpu.hip
	 * duplex_setup): 64 CUs every 4th, 64 contiguous, 128 every 2nd */
	int ncu = 0;
	CHECK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
	auto masked = [&](int pick, int mod, int lim) {
		uint32_t m[64] = { 0 };
		int got = 0;
		for (int c = 0; c < ncu && got < lim; c++)
			if (c % mod == pick) {
				m[c / 32] |= 1u << (c % 32);
				got++;
			}
		hipStream_t st;
		CHECK(hipExtStreamCreateWithCUMask(&st, (uint32_t)(ncu + 31) / 32, m));
		return st;
	};
	hipStream_t s_m4 = masked(0, 4, 64), s_m1 = masked(0, 1, 64), s_m2 = masked(0, 2, 128),
	    s_m8 = masked(0, 8, 32);
	printf("{\"cus\": %d}\n", ncu);
	struct cs { const char *name; bool ring, host, h2d, direct; int mask = 0; };
	const cs cases[] = {
		{ "linear", false, false, false, false },
		{ "ring", true, false, false, false },
		{ "ring_host", true, true, false, false },
		{ "ring_h2d", true, false, true, false },
		{ "ring_host_h2d", true, true, true, false },
		{ "linear_h2d", false, false, true, false },
		/* the pageable output registered for the run, written directly */
		{ "direct_h2d", false, false, true, true },
		{ "direct", false, false, false, true },
		{ "direct_h2d_cus64_every4th", false, false, true, true, 4 },
		{ "direct_h2d_cus64_first", false, false, true, true, 1 },
		{ "direct_h2d_cus128_every2nd", false, false, true, true, 2 },
		{ "direct_h2d_cus32_every8th", false, false, true, true, 8 },
		{ "direct_cus64_every4th", false, false, false, true, 4 },
	};
	for (int rep = 0; rep < 2; rep++)
	for (const cs &c : cases) {
		std::vector<double> ms;
		for (int it = 0; it < 6; it++) {
			CHECK(hipDeviceSynchronize());
			const double t0 = now_ms();
			bool reg = false;
			if (c.h2d) {
				reg = hipHostRegister(h_in, IN_BYTES, hipHostRegisterDefault) ==
				    hipSuccess;
				for (int k = 0; k < NSLAB; k++)
					CHECK(hipMemcpyAsync(d_in + k * (IN_BYTES / NSLAB),
					    h_in + k * (IN_BYTES / NSLAB), IN_BYTES / NSLAB,
					    hipMemcpyHostToDevice, s_in));
			}
			uint8_t *d_dir = NULL;
			double t_reg = 0.0;
			if (c.direct) {
				const double r0 = now_ms();
				CHECK(hipHostRegister(h_dst, NSLAB * SLAB, hipHostRegisterDefault));
				CHECK(hipHostGetDevicePointer((void **)&d_dir, h_dst, 0));
				t_reg = now_ms() - r0;
			}
			auto issue = [&](int k) {
				uint8_t *dst = c.direct ? d_dir + k * SLAB : c.ring ?
				    d_ring + (k % SLOTS) * SLAB : d_lin + k * SLAB;
				hipStream_t so = c.mask == 4 ? s_m4 : c.mask == 1 ? s_m1 :
				    c.mask == 2 ? s_m2 : c.mask == 8 ? s_m8 : s_out;
				hipLaunchKernelGGL(k_slab_out, dim3(128), dim3(256), 0, so,
				    (const uint4 *)(d_src + k * SLAB), (uint4 *)dst,
				    (uint64_t)(SLAB / 16));
				CHECK(hipEventRecord(ev[k], so));
			};
			for (int k = 0; k < SLOTS; k++)
				issue(k);
			for (int k = 0; k < NSLAB; k++) {
				CHECK(hipEventSynchronize(ev[k]));
				if (c.host) {
					const uint8_t *from = c.ring ? h_ring + (k % SLOTS) * SLAB :
					    h_lin + k * SLAB;
					std::vector<xa_pool::piece> p(1, xa_pool::piece{
					    h_dst + k * SLAB, from, SLAB });
					pool.run(p);
				}
				if (k + SLOTS < NSLAB)
					issue(k + SLOTS);
			}
			CHECK(hipStreamSynchronize(s_in));
			const double t = now_ms() - t0;
			if (reg)
				CHECK(hipHostUnregister(h_in));
			if (c.direct) {
				CHECK(hipHostUnregister(h_dst));
				if (it == 1 || it == 5)
					printf("  (register 256 MiB: %.3f ms)\n", t_reg);
			}
			if (it >= 1)
				ms.push_back(t);
		}
		std::sort(ms.begin(), ms.end());
		printf("{\"rep\": %d, \"case\": \"%s\", \"ms\": %.3f, \"out_GBps\": %.1f}\n",
		    rep, c.name, ms[ms.size() / 2], NSLAB * SLAB / ms[ms.size() / 2] / 1e6);
		fflush(stdout);
	}
	return 0;
}
