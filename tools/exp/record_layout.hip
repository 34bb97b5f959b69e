// The lane analysis' record copy (k_ana.hip: EncAna's 5,088-byte live
// prefix in and out of the lane's private segment) by record layout, at the
// headline's 262,144 channels:
//   aos      the engine's layout: one 17,872-byte EncState per channel, the
//            prefix at offset 11,024; lane g copies channel perm[g]'s prefix
//            with 16-byte loads / stores (lane_copy_x4), as k_enc_ana does
//   soa      channel-interleaved in lane order: dword d of lane slot g at
//            [d][g], so each copy instruction moves 256 contiguous bytes of
//            the wave (dword loads / stores)
//   gather / scatter   what the interleaved layout costs around the lane
//            kernel when the records stay per channel (checkpoint / import
//            and the NPP kernel read them per channel): the prefixes of
//            perm[g] moved into / out of slot g, coalesced on the
//            interleaved side through an LDS transpose
// Each lane kernel holds the copy in its private segment and touches every
// dword (xor into a checksum) so nothing is dropped.  perm: identity, or the
// pitch-class order's scatter approximated by a random permutation.
//   hipcc -O3 --offload-arch=gfx950 tools/exp/record_layout.hip -o /tmp/rl && /tmp/rl
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <stdint.h>

#define N 262144
#define REC_STRIDE 17872
#define REC_OFF 11024
#define LIVE 5088
#define LW (LIVE / 4)	/* 1272 dwords */
#define L4 (LIVE / 16)	/* 318 x 16 bytes */

typedef uint32_t v4u __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(64, 4) void k_aos(uint8_t *rec, const int *perm, uint32_t *sum)
{
	const int g = blockIdx.x * 64 + threadIdx.x;
	const int c = perm[g];
	v4u p[L4];
	const v4u *s = (const v4u *) (rec + (size_t) c * REC_STRIDE + REC_OFF);
#pragma unroll 8
	for (int i = 0; i < L4; i++)
		p[i] = s[i];
	uint32_t x = 0;
	for (int i = 0; i < L4; i++) {
		p[i].x ^= (uint32_t) i;
		x ^= p[i].x ^ p[i].y ^ p[i].z ^ p[i].w;
	}
	v4u *d = (v4u *) (rec + (size_t) c * REC_STRIDE + REC_OFF);
#pragma unroll 8
	for (int i = 0; i < L4; i++)
		d[i] = p[i];
	sum[g] = x;
}

__global__ __launch_bounds__(64, 4) void k_soa(uint32_t *il, uint32_t *sum)
{
	const int g = blockIdx.x * 64 + threadIdx.x;
	uint32_t p[LW];
#pragma unroll 8
	for (int i = 0; i < LW; i++)
		p[i] = il[(size_t) i * N + g];
	uint32_t x = 0;
	for (int i = 0; i < LW; i++) {
		p[i] ^= (uint32_t) i;
		x ^= p[i];
	}
#pragma unroll 8
	for (int i = 0; i < LW; i++)
		il[(size_t) i * N + g] = p[i];
	sum[g] = x;
}

/* slot g's prefix <- channel perm[g]'s (DIR 0) or back (DIR 1); a workgroup
 * of 256 threads moves 64 slots: each wave streams 16 records' 5 KB row
 * ways through LDS in blocks of 64 dwords */
template <int DIR>
__global__ __launch_bounds__(256) void k_move(uint8_t *rec, uint32_t *il, const int *perm)
{
	__shared__ uint32_t t[64][65];
	const int g0 = blockIdx.x * 64, w = threadIdx.x / 64, l = threadIdx.x % 64;
	for (int d0 = 0; d0 < LW; d0 += 64) {
		const int nd = LW - d0 < 64 ? LW - d0 : 64;
		if (DIR == 0) {
			for (int r = w; r < 64; r += 4) {
				const uint32_t *s = (const uint32_t *) (rec + (size_t) perm[g0 + r] * REC_STRIDE + REC_OFF);
				if (l < nd)
					t[r][l] = s[d0 + l];
			}
			__syncthreads();
			for (int d = w; d < nd; d += 4)
				il[(size_t) (d0 + d) * N + g0 + l] = t[l][d];
		} else {
			for (int d = w; d < nd; d += 4)
				t[l][d] = il[(size_t) (d0 + d) * N + g0 + l];
			__syncthreads();
			for (int r = w; r < 64; r += 4) {
				uint32_t *s = (uint32_t *) (rec + (size_t) perm[g0 + r] * REC_STRIDE + REC_OFF);
				if (l < nd)
					s[d0 + l] = t[r][l];
			}
		}
		__syncthreads();
	}
}

static float time_it(void (*f)(void *), void *a, int reps)
{
	hipEvent_t e0, e1;
	hipEventCreate(&e0);
	hipEventCreate(&e1);
	f(a);
	hipDeviceSynchronize();
	hipEventRecord(e0);
	for (int i = 0; i < reps; i++)
		f(a);
	hipEventRecord(e1);
	hipEventSynchronize(e1);
	float ms;
	hipEventElapsedTime(&ms, e0, e1);
	return ms / reps;
}

struct Args {
	uint8_t *rec;
	uint32_t *il, *sum;
	int *perm;
};

static void run_aos(void *p)
{
	Args *a = (Args *) p;
	k_aos<<<N / 64, 64>>>(a->rec, a->perm, a->sum);
}
static void run_soa(void *p)
{
	Args *a = (Args *) p;
	k_soa<<<N / 64, 64>>>(a->il, a->sum);
}
static void run_gather(void *p)
{
	Args *a = (Args *) p;
	k_move<0><<<N / 64, 256>>>(a->rec, a->il, a->perm);
}
static void run_scatter(void *p)
{
	Args *a = (Args *) p;
	k_move<1><<<N / 64, 256>>>(a->rec, a->il, a->perm);
}

int main()
{
	Args a;
	hipMalloc(&a.rec, (size_t) N * REC_STRIDE);
	hipMalloc(&a.il, (size_t) N * LIVE);
	hipMalloc(&a.sum, sizeof(uint32_t) * N);
	hipMalloc(&a.perm, sizeof(int) * N);
	hipMemset(a.rec, 1, (size_t) N * REC_STRIDE);
	hipMemset(a.il, 2, (size_t) N * LIVE);
	int *h = (int *) malloc(sizeof(int) * N);
	for (int order = 0; order < 2; order++) {
		for (int i = 0; i < N; i++)
			h[i] = i;
		if (order)
			for (int i = N - 1; i > 0; i--) {
				int j = (int) (((uint64_t) rand() * 2654435761u) % (uint64_t) (i + 1));
				int t = h[i];
				h[i] = h[j];
				h[j] = t;
			}
		hipMemcpy(a.perm, h, sizeof(int) * N, hipMemcpyHostToDevice);
		const char *on = order ? "random" : "identity";
		printf("{\"perm\": \"%s\", \"aos_copy_ms\": %.3f, \"soa_copy_ms\": %.3f, \"gather_ms\": %.3f, "
		       "\"scatter_ms\": %.3f}\n",
		       on, time_it(run_aos, &a, 5), time_it(run_soa, &a, 5), time_it(run_gather, &a, 5),
		       time_it(run_scatter, &a, 5));
	}
	return 0;
}
