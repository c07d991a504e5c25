/*
 * dep_probe.hip -- do two CU-masked streams overlap when one waits on the
 * other?  (The duplex decode's slab kernels and its copy-out ran strictly one
 * after the other in the kernel trace even on disjoint CU masks, R6-7.)
 *
 * Per slab k: a "decode" stand-in on s_dec (an HBM -> HBM copy of 96 MiB,
 * ~50 us, 192 CUs) and a copy-out on s_out (16 MiB HBM -> pinned host, ~0.31
 * ms, 64 CUs) that must follow decode k.  All 16 slabs issued up front.
 *   none    no dependency at all (the overlap ceiling)
 *   event   hipEventRecord on s_dec, hipStreamWaitEvent on s_out (as the route)
 *   value   hipStreamWriteValue32 of k+1 on s_dec, hipStreamWaitValue32 >= k+1
 *           on s_out (a queue-level wait on a device word, no event)
 *   ahead   event, but each copy-out waits for decode k+3's event instead,
 *           as if every decode were long done
 *   gated   event, issued as the route issues: slabs 0-3 up front, slab k+4
 *           once the host has seen copy-out k end (hipEventSynchronize)
 *   gated_dec_ahead  every decode issued up front, only the copy-outs gated
 *   gated_value      gated, with the value wait instead of the event
 * Median of 5 runs of the whole 16-slab sequence.
 *
 * build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -o tools/bin/dep_probe \
 *            tools/dep_probe.hip
 */
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <algorithm>
#include <chrono>
#include <vector>

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
	fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); exit(1); } } while (0)

#define SLAB	((size_t)16 << 20)
#define DEC	((size_t)96 << 20)
#define NSLAB	16

__global__ __launch_bounds__(256) void
k_copy(const uint4 *src, uint4 *dst, uint64_t n16)
{
	for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n16;
	    i += (uint64_t)gridDim.x * 256u)
		dst[i] = src[i];
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
	int ncu = 0;
	CHECK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
	int wv = 0;
	(void)hipDeviceGetAttribute(&wv, hipDeviceAttributeCanUseStreamWaitValue, 0);
	uint32_t mo[64] = { 0 }, md[64] = { 0 };
	for (int c = 0; c < ncu; c++)
		((c % 4 == 0 && c / 4 < 64) ? mo : md)[c / 32] |= 1u << (c % 32);
	hipStream_t s_out, s_dec;
	CHECK(hipExtStreamCreateWithCUMask(&s_out, (uint32_t)(ncu + 31) / 32, mo));
	CHECK(hipExtStreamCreateWithCUMask(&s_dec, (uint32_t)(ncu + 31) / 32, md));
	uint8_t *a, *b, *src, *h, *d_h;
	uint32_t *flag;
	CHECK(hipMalloc(&a, DEC));
	CHECK(hipMalloc(&b, DEC));
	CHECK(hipMalloc(&src, NSLAB * SLAB));
	CHECK(hipMalloc(&flag, 64));
	CHECK(hipMemset(a, 1, DEC));
	CHECK(hipMemset(src, 2, NSLAB * SLAB));
	CHECK(hipHostMalloc((void **)&h, NSLAB * SLAB, hipHostMallocDefault));
	CHECK(hipHostGetDevicePointer((void **)&d_h, h, 0));
	std::vector<hipEvent_t> ev(NSLAB);
	for (hipEvent_t &e : ev)
		CHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
	printf("{\"cus\": %d, \"can_wait_value\": %d}\n", ncu, wv);
	std::vector<hipEvent_t> eo(NSLAB);
	for (hipEvent_t &e : eo)
		CHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
	const char *modes[] = { "none", "event", "value", "ahead", "gated",
	    "gated_dec_ahead", "gated_value" };
	for (int rep = 0; rep < 2; rep++)
	for (int m = 0; m < 7; m++) {
		if (m >= 4) {
			std::vector<double> ms;
			for (int it = 0; it < 6; it++) {
				CHECK(hipMemset(flag, 0, 64));
				CHECK(hipDeviceSynchronize());
				const double t0 = now_ms();
				auto dec = [&](int k) {
					hipLaunchKernelGGL(k_copy, dim3(768), dim3(256), 0, s_dec,
					    (const uint4 *)a, (uint4 *)b, (uint64_t)(DEC / 16));
					if (m == 6)
						CHECK(hipStreamWriteValue32(s_dec, flag,
						    (uint32_t)k + 1u, 0));
					else
						CHECK(hipEventRecord(ev[k], s_dec));
				};
				auto out = [&](int k) {
					if (m == 6)
						CHECK(hipStreamWaitValue32(s_out, flag, (uint32_t)k + 1u,
						    hipStreamWaitValueGte, 0xffffffffu));
					else
						CHECK(hipStreamWaitEvent(s_out, ev[k], 0));
					hipLaunchKernelGGL(k_copy, dim3(128), dim3(256), 0, s_out,
					    (const uint4 *)(src + k * SLAB),
					    (uint4 *)(d_h + k * SLAB), (uint64_t)(SLAB / 16));
					CHECK(hipEventRecord(eo[k], s_out));
				};
				if (m == 5)
					for (int k = 0; k < NSLAB; k++)
						dec(k);
				for (int k = 0; k < 4; k++) {
					if (m != 5)
						dec(k);
					out(k);
				}
				for (int k = 0; k < NSLAB; k++) {
					CHECK(hipEventSynchronize(eo[k]));
					if (k + 4 < NSLAB) {
						if (m != 5)
							dec(k + 4);
						out(k + 4);
					}
				}
				CHECK(hipStreamSynchronize(s_out));
				CHECK(hipStreamSynchronize(s_dec));
				if (it >= 1)
					ms.push_back(now_ms() - t0);
			}
			std::sort(ms.begin(), ms.end());
			printf("{\"rep\": %d, \"mode\": \"%s\", \"ms\": %.3f}\n", rep,
			    modes[m], ms[ms.size() / 2]);
			fflush(stdout);
			continue;
		}
		if (m == 2 && !wv)
			continue;
		std::vector<double> ms;
		for (int it = 0; it < 6; it++) {
			CHECK(hipMemset(flag, 0, 64));
			CHECK(hipDeviceSynchronize());
			const double t0 = now_ms();
			for (int k = 0; k < NSLAB; k++) {
				hipLaunchKernelGGL(k_copy, dim3(768), dim3(256), 0, s_dec,
				    (const uint4 *)a, (uint4 *)b, (uint64_t)(DEC / 16));
				if (m == 1 || m == 3)
					CHECK(hipEventRecord(ev[k], s_dec));
				if (m == 2)
					CHECK(hipStreamWriteValue32(s_dec, flag, (uint32_t)k + 1u, 0));
			}
			for (int k = 0; k < NSLAB; k++) {
				if (m == 1)
					CHECK(hipStreamWaitEvent(s_out, ev[k], 0));
				if (m == 3 && k >= 3)
					CHECK(hipStreamWaitEvent(s_out, ev[k - 3], 0));
				if (m == 2)
					CHECK(hipStreamWaitValue32(s_out, flag, (uint32_t)k + 1u,
					    hipStreamWaitValueGte, 0xffffffffu));
				hipLaunchKernelGGL(k_copy, dim3(128), dim3(256), 0, s_out,
				    (const uint4 *)(src + k * SLAB), (uint4 *)(d_h + k * SLAB),
				    (uint64_t)(SLAB / 16));
			}
			CHECK(hipStreamSynchronize(s_out));
			CHECK(hipStreamSynchronize(s_dec));
			if (it >= 1)
				ms.push_back(now_ms() - t0);
		}
		std::sort(ms.begin(), ms.end());
		printf("{\"rep\": %d, \"mode\": \"%s\", \"ms\": %.3f}\n", rep, modes[m],
		    ms[ms.size() / 2]);
		fflush(stdout);
	}
	return 0;
}
