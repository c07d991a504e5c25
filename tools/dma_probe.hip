// Probe the LDS layout of global_load_lds at 12 and 16 bytes per lane
// (gfx950): one wave, lane t reads `size` bytes at src + off0 + t*size,
// then the first 1280 LDS bytes are dumped.  Prints, per size, the first
// LDS byte offset that differs from the packed layout (base + t*size).
//   hipcc --offload-arch=gfx950 -O2 -o build/dma_probe tools/dma_probe.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

#define LDS_PTR(p) ((__attribute__((address_space(3))) void *)(p))

template <int S>
__global__ void probe(const uint8_t *src, uint8_t *out, int off0)
{
	__shared__ __attribute__((aligned(16))) uint8_t lds[1280];
	for (int i = threadIdx.x; i < 1280; i += 64)
		lds[i] = 0xEE;
	__syncthreads();
	if (S == 12)
		__builtin_amdgcn_global_load_lds(src + off0 + threadIdx.x * S,
		    LDS_PTR(lds), 12, 0, 0);
	else
		__builtin_amdgcn_global_load_lds(src + off0 + threadIdx.x * S,
		    LDS_PTR(lds), 16, 0, 0);
	asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
	__syncthreads();
	for (int i = threadIdx.x; i < 1280; i += 64)
		out[i] = lds[i];
}

static int check(int size, int off0, const uint8_t *h)
{
	for (int i = 0; i < 64 * size; i++)
		if (h[i] != (uint8_t)(off0 + i)) {
			printf("size %d off0 %d: packed layout breaks at LDS byte %d "
			    "(got %u want %u); first 40: ", size, off0, i, h[i],
			    (uint8_t)(off0 + i));
			for (int k = 0; k < 40; k++)
				printf("%u ", h[k]);
			printf("\n");
			return 1;
		}
	printf("size %d off0 %d: packed (base + lane*%d)\n", size, off0, size);
	return 0;
}

int main()
{
	uint8_t *src, *out, h[1280], hs[4096];
	for (int i = 0; i < 4096; i++)
		hs[i] = (uint8_t)i;
	if (hipMalloc(&src, 4096) || hipMalloc(&out, 1280))
		return 2;
	(void)hipMemcpy(src, hs, 4096, hipMemcpyHostToDevice);
	int bad = 0;
	for (int off0 : {0, 4, 8}) {
		probe<12><<<1, 64>>>(src, out, off0);
		(void)hipMemcpy(h, out, 1280, hipMemcpyDeviceToHost);
		bad |= check(12, off0, h);
		probe<16><<<1, 64>>>(src, out, off0);
		(void)hipMemcpy(h, out, 1280, hipMemcpyDeviceToHost);
		bad |= check(16, off0, h);
	}
	return bad;
}
