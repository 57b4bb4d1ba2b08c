# r06 experiment: per-workgroup s_memrealtime stamps for the coarse-head patch
# (tools/build_head_variant.sh with STAMPS=1 applies it; tools/head_probe.py reads them).
p = "csrc/dis_search8.hip"; s = open(p).read()
old = "typedef __attribute__((address_space(1))) int g_i32;"
assert old in s
s = s.replace(old, """__shared__ unsigned long long s_tw;
__device__ unsigned long long g_ts[16384 * 4];
__device__ unsigned int g_ts_n;
""" + old, 1)
old = """        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }"""
assert old in s
s = s.replace(old, """        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        s_tw = __builtin_amdgcn_s_memrealtime();
    }""", 1)
old = """    if (threadIdx.x == 0) ticket = atomicAdd(h.ticket, 1);
    __syncthreads();"""
assert old in s
s = s.replace(old, """    unsigned long long t0 = 0;
    if (threadIdx.x == 0) { ticket = atomicAdd(h.ticket, 1); t0 = __builtin_amdgcn_s_memrealtime(); s_tw = t0; }
    __syncthreads();""", 1)
old = """    if (threadIdx.x == 0) __hip_atomic_fetch_add((g_i32*)(done + j), 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}"""
assert old in s
s = s.replace(old, """    if (threadIdx.x == 0) {
        const unsigned long long te = __builtin_amdgcn_s_memrealtime();
        __hip_atomic_fetch_add((g_i32*)(done + j), 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const unsigned slot = atomicAdd(&g_ts_n, 1u);
        if (slot < 16384) {
            g_ts[slot * 4 + 0] = (unsigned long long)j | ((((unsigned long long)(uintptr_t)h.ticket) >> 5 & 7) << 8);
            g_ts[slot * 4 + 1] = t0;
            g_ts[slot * 4 + 2] = s_tw;
            g_ts[slot * 4 + 3] = te;
        }
    }
}""", 1)
s += """
extern "C" int dis_head_stamps(void* dst, int maxn)
{
    unsigned n = 0, z = 0;
    if (hipMemcpyFromSymbol(&n, HIP_SYMBOL(dis::g_ts_n), 4) != hipSuccess) return -1;
    if ((int)n > maxn) n = maxn;
    if (n > 16384) n = 16384;
    if (n && hipMemcpyFromSymbol(dst, HIP_SYMBOL(dis::g_ts), (size_t)n * 32) != hipSuccess) return -2;
    if (hipMemcpyToSymbol(HIP_SYMBOL(dis::g_ts_n), &z, 4) != hipSuccess) return -3;
    return (int)n;
}
"""
open(p, "w").write(s)
