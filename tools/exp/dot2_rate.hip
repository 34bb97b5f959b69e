// issue-rate microbenchmark: v_dot2c_i32_i16 vs plain 32-bit VALU (one wave
// per SIMD and four), 16 independent accumulators per lane
#include <hip/hip_runtime.h>
#include <stdio.h>
typedef short v2s __attribute__((ext_vector_type(2)));
template <int MODE>
__global__ void k(const unsigned *in, int *out, int iters)
{
	unsigned a = in[threadIdx.x], b = in[threadIdx.x + 64];
	int acc[16];
	for (int i = 0; i < 16; i++) acc[i] = in[i] ;
	for (int it = 0; it < iters; it++) {
#pragma unroll
		for (int i = 0; i < 16; i++) {
			if (MODE == 0)
				acc[i] = __builtin_amdgcn_sdot2(__builtin_bit_cast(v2s, a + i), __builtin_bit_cast(v2s, b), acc[i], false);
			else if (MODE == 1)
				acc[i] = acc[i] + (int)(a ^ i);
			else
				acc[i] = __builtin_amdgcn_sdot2(__builtin_bit_cast(v2s, a), __builtin_bit_cast(v2s, b + i), acc[i], false) ;
		}
		a = a * 3 + 1;
	}
	int s = 0;
	for (int i = 0; i < 16; i++) s += acc[i];
	out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
int main()
{
	unsigned *in; int *out;
	hipMalloc(&in, 4096); hipMalloc(&out, 1 << 24);
	hipMemset(in, 1, 4096);
	hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
	const int iters = 20000;
	for (int wps = 1; wps <= 4; wps *= 4) {
		int blocks = 256 * 4 * wps;	// waves = blocks (64 threads each)
		for (int mode = 0; mode < 3; mode++) {
			for (int rep = 0; rep < 2; rep++) {
				hipEventRecord(e0);
				if (mode == 0) k<0><<<blocks, 64>>>(in, out, iters);
				else if (mode == 1) k<1><<<blocks, 64>>>(in, out, iters);
				else k<2><<<blocks, 64>>>(in, out, iters);
				hipEventRecord(e1); hipEventSynchronize(e1);
				float ms; hipEventElapsedTime(&ms, e0, e1);
				double instr = 16.0 * iters;	// per wave, of the measured kind
				double cyc = ms * 1e-3 * 2.4e9;	// wall cycles at 2.4 GHz
				if (rep) printf("waves/SIMD %d mode %d: %.3f ms, %.2f cycles per instr per SIMD\n", wps, mode, ms, cyc / (instr * wps));
			}
		}
	}
	return 0;
}
