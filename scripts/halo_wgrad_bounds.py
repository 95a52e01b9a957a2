# Host-side replay of conv3x3s1_halo_wgrad_kernel's index math (csrc/kernels/conv_halo.hip):
# for every ResNet-18 stride-1 3x3 shape and chunk plan, asserts that every dY / X load and
# every LDS halo read stays in bounds.  Run: python scripts/halo_wgrad_bounds.py
# host-side bounds check of conv3x3s1_halo_wgrad_kernel's index math
SLOTS, MAXPOS = 224, 360
def wp(W): return (W + 7) & ~7
def ok(H, W, Cin, Cout):
    Wp = wp(W); R = SLOTS // Wp
    if SLOTS % Wp: return False
    Hs = H if H < R else R
    return (R // Hs) * (Hs + 2) * (Wp + 2) <= MAXPOS and Cin % 32 == 0 and Cout % 64 == 0
def quantum(H, W):
    R = SLOTS // wp(W); return H if H < R else 1
def plan(N, H, W, Cin, Cout, target=256):
    bpc = (Cout // 64) * (Cin // 32); chunks = max(1, target // bpc)
    rows = N * H; rpc = -(-rows // chunks); q = quantum(H, W); rpc = -(-rpc // q) * q
    return rpc
def check(N, H, W, Cin, Cout, rpc):
    Wp = wp(W); R = SLOTS // Wp; XW = Wp + 2
    Hs = H if H < R else R; nimg = R // Hs; live = nimg * Hs
    nxc = nimg * (Hs + 2) * XW * 4
    assert nxc <= 6 * 256, nxc
    rows = N * H; chunks = -(-rows // rpc)
    for z in range(chunks):
        rbeg = z * rpc; rend = min(rows, rbeg + rpc)
        def grp(r): return min(live if H < R else min(R, H - r % H), rend - r)
        r0 = rbeg; cnt = grp(r0) if r0 < rend else 0
        while cnt > 0:
            if H < R: assert r0 % H == 0, (r0, H)
            for slot in range(SLOTS):
                rr, col = divmod(slot, Wp)
                if rr < cnt and col < W:
                    fr = r0 + rr; assert 0 <= fr < rows
            for c in range(nxc):
                pos, _ = divmod(c, 4); hr, cc = divmod(pos, XW)
                k, loc = divmod(hr, Hs + 2); fr = r0 + k * Hs
                n = fr // H; hh = fr - n * H - 1 + loc; ww = cc - 1
                if k * Hs < cnt and 0 <= hh < H and 0 <= ww < W:
                    assert 0 <= n < N, (n, N); 
            # MFMA LDS rows stay in the staged halo
            for s in range(SLOTS):
                r = min(s // Wp, live - 1); hrow = r + 2 * (r // Hs)
                for kh in range(3):
                    assert (hrow + kh) * XW + (s % Wp) + 2 < nimg * (Hs + 2) * XW, (s, kh)
            r0 += cnt; cnt = grp(r0) if r0 < rend else 0
    return chunks
cases = [(2,56,64,64,4),(2,56,64,64,12),(3,28,128,64,8),(3,28,64,128,24),(2,14,256,64,16),(4,7,64,512,14),(8,7,64,64,21)]
for N,H,Cin,Cout,rpc in cases:
    assert ok(H,H,Cin,Cout); check(N,H,H,Cin,Cout,rpc); check(N,H,H,Cin,Cout,plan(N,H,H,Cin,Cout)); check(N,H,H,Cin,Cout,N*H)
for N in (8, 7, 32, 5, 3):
    for H,C in ((56,64),(28,128),(14,256),(7,512),(16,64),(8,128),(4,256),(2,512),(32,64)):
        if ok(H,H,C,C):
            ch = check(N,H,H,C,C,plan(N,H,H,C,C)); print(N,H,C,'rpc',plan(N,H,H,C,C),'chunks',ch)
print("all in bounds")
