# r06 experiment (not kept): k_vr_lin tiles in a chunked XCD order (each XCD
# a run of R = 8 tiles along x). Run in the package directory of a /tmp copy of the tree.
p = "csrc/dis_varref.hip"; s = open(p).read()
old = """    const int W = L.W, H = L.H, pr = blockIdx.z, tid = threadIdx.x;
    const int x0 = blockIdx.x * kLW, y0 = blockIdx.y * kLH;"""
assert old in s
new = """    const int W = L.W, H = L.H, tid = threadIdx.x;
    int tx, ty, pr;
    {
        constexpr int R = 8;
        const int nbx = gridDim.x, nby = gridDim.y, nb = nbx * nby * gridDim.z;
        const int lin = blockIdx.x + nbx * (blockIdx.y + nby * blockIdx.z);
        const int full = nb / (8 * R) * (8 * R);
        int t = lin;
        if (lin < full) {
            const int x = lin % 8, m = lin / 8;
            t = ((m / R) * 8 + x) * R + m % R;
        }
        tx = __builtin_amdgcn_readfirstlane(t % nbx);
        ty = __builtin_amdgcn_readfirstlane((t / nbx) % nby);
        pr = __builtin_amdgcn_readfirstlane(t / (nbx * nby));
    }
    const int x0 = tx * kLW, y0 = ty * kLH;"""
s = s.replace(old, new, 1); open(p, "w").write(s)
