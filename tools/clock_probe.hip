/*
 * clock_probe.hip -- the shader clock the GPU runs at, read from inside a
 * kernel: one wave counts s_memtime (shader-clock counter) against
 * s_memrealtime (the constant 100 MHz counter) over `ticks` ticks of the
 * latter, and stores {d_memtime, d_realtime} with a vector store.  MHz =
 * d_memtime / d_realtime * 100.  Loaded by tools/clock_probe.py through
 * ctypes (clk_launch), on the stream the decodes run on, so that it reads
 * the clock right after whatever ran (or did not run) before it.
 *
 * build: hipcc --offload-arch=gfx950 -O3 -fPIC -shared -o tools/bin/clock_probe.so \
 *            tools/clock_probe.hip
 */
#include <hip/hip_runtime.h>
#include <stdint.h>

__global__ __launch_bounds__(64) void
clk_kernel(uint64_t *out, uint32_t ticks)
{
	const uint64_t r0 = __builtin_amdgcn_s_memrealtime();
	const uint64_t c0 = __builtin_amdgcn_s_memtime();
	uint64_t r1 = r0, c1 = c0;
	while (r1 - r0 < ticks) {
		__builtin_amdgcn_s_sleep(1);
		r1 = __builtin_amdgcn_s_memrealtime();
		c1 = __builtin_amdgcn_s_memtime();
	}
	if (threadIdx.x == 0) {
		out[0] = c1 - c0;
		out[1] = r1 - r0;
	}
}

extern "C" int
clk_launch(void *out, uint32_t ticks, void *stream)
{
	hipLaunchKernelGGL(clk_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream,
	    (uint64_t *)out, ticks);
	return hipGetLastError() == hipSuccess ? 0 : -1;
}
