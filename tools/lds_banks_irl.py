"""LDS bank model of irl_kernel (kernels/irl.hip) per MI355X_MICROARCH.md §LDS: LDS-array cycles per
chunk step of its three bank-sensitive accesses -- the expand epilogue's stores into the padded
planes, the depthwise row tasks' window reads, and their stores into the depthwise tile -- for the
current layout and for padded plane rows (PW), plane strides (PPs) and tile channel strides.

    python tools/lds_banks_irl.py
"""
import itertools

from lds_banks import GROUPS, DWORDS, cycles

# ds_read2_b64: two accesses, each 4 x 16 contiguous lanes, banks mod 32
GROUPS["r2b64"] = ([list(range(16 * i, 16 * i + 16)) for i in range(4)], 32)
DWORDS["r2b64"] = 2
GROUPS["b32w"] = ([list(range(0, 32)), list(range(32, 64))], 32)
DWORDS["b32w"] = 1

CEC = 16


def geometry(K, HW, S, NI):
    HO = HW // S
    P, PO = HW * HW, HO * HO
    PL = K // 2 if S == 1 else K // 2 - 1
    PH = (HO - 1) * S + K
    PW = (PH + 1) & ~1
    NE = (P + 15) // 16
    NET = NI * NE
    NEW = (NET + 3) // 4
    NCT = (PO + 31) // 32
    NCP = NCT * 32
    RW = HO // 2 if CEC * HO * 2 <= 256 and HO % 2 == 0 else HO
    RPR = HO // RW
    WWIN = ((RW - 1) * S + K + 1) & ~1
    NTASK = CEC * HO * RPR
    return dict(HO=HO, P=P, PO=PO, PL=PL, PH=PH, PW=PW, NE=NE, NET=NET, NEW=NEW, NCP=NCP, RW=RW, RPR=RPR,
                WWIN=WWIN, NTASK=NTASK)


def model(K, HW, S, NI, PW=None, PPs=None, DCs=None, read=None):
    g = geometry(K, HW, S, NI)
    PW = PW or g["PW"]
    PPs = PPs or g["PH"] * PW
    DCs = DCs or NI * g["NCP"]
    HO, P, PL, NE, NET, NEW, RW, RPR, NTASK = (g[k] for k in ("HO", "P", "PL", "NE", "NET", "NEW", "RW", "RPR", "NTASK"))
    res = {}
    # expand epilogue: ds_write_b32 per r (4 channels of a lane)
    cyc = ideal = 0
    for mw in range(4):
        for i in range(NEW):
            t = mw + 4 * i
            if t >= NET:
                continue
            for r in range(4):
                addr = []
                for lane in range(64):
                    col, kq = lane & 15, lane >> 4
                    j = t // NE
                    p = (t - j * NE) * 16 + col
                    if p >= P:
                        addr.append(None)
                        continue
                    y, x = p // HW, p % HW
                    addr.append((j * CEC + 4 * kq + r) * PPs + (y + PL) * PW + x + PL)
                cyc += cycles("b32w", addr)
                ideal += 2
    res["expand_store"] = (cyc, ideal)
    # depthwise window reads
    kinds = [read] if read else ["b64r", "r2b64", "b128r"]
    for kind in kinds:
        vw = DWORDS[kind] if kind != "r2b64" else 2
        cyc = ideal = 0
        nread = (g["WWIN"] + vw - 1) // vw
        for w in range(4):
            for ky in range(K):
                for e in range(nread):
                    addr = []
                    for lane in range(64):
                        dt = w * 64 + lane
                        if dt >= NI * NTASK:
                            addr.append(None)
                            continue
                        dj, dtj = dt // NTASK, dt % NTASK
                        dc, dr = dtj // (HO * RPR), dtj % (HO * RPR)
                        dy, dx0 = dr // RPR, (dr % RPR) * RW
                        addr.append((dj * CEC + dc) * PPs + dx0 * S + (dy * S + ky) * PW + vw * e)
                    cyc += cycles(kind, addr)
                    ideal += len(GROUPS[kind][0])
        res["dw_read_" + kind] = (cyc, ideal)
    # depthwise tile stores (b32 per output)
    cyc = ideal = 0
    for w in range(4):
        for o in range(RW):
            addr = []
            for lane in range(64):
                dt = w * 64 + lane
                if dt >= NI * NTASK:
                    addr.append(None)
                    continue
                dj, dtj = dt // NTASK, dt % NTASK
                dc, dr = dtj // (HO * RPR), dtj % (HO * RPR)
                dy, dx0 = dr // RPR, (dr % RPR) * RW
                addr.append(dc * DCs + dj * g["NCP"] + dy * HO + dx0 + o)
            cyc += cycles("b32w", addr)
            ideal += 2
    res["dw_store"] = (cyc, ideal)
    return g, res


INST = [(3, 14, 1, 1), (5, 14, 1, 1), (5, 14, 2, 1), (5, 14, 2, 2), (5, 7, 1, 1), (5, 7, 1, 2)]

if __name__ == "__main__":
    for K, HW, S, NI in INST:
        g, r = model(K, HW, S, NI)
        print(f"irl<{K},{HW},{S},NI={NI}> PW {g['PW']} PP {g['PH'] * g['PW']} RW {g['RW']} WWIN {g['WWIN']}: " +
              ", ".join(f"{k} {c}/{i}" for k, (c, i) in r.items()))
        # search: row pitch, plane stride pad, tile channel stride pad
        best = {}
        for pw, pp, dc in itertools.product(range(g["PW"], g["PW"] + 16, 2), range(0, 64, 4), range(0, 32, 4)):
            _, rr = model(K, HW, S, NI, PW=pw, PPs=g["PH"] * pw + pp, DCs=NI * g["NCP"] + dc)
            for kind in ("b64r", "r2b64", "b128r"):
                tot = rr["expand_store"][0] + rr["dw_read_" + kind][0] + rr["dw_store"][0]
                if kind not in best or tot < best[kind][0]:
                    best[kind] = (tot, pw, pp, dc, rr["expand_store"][0], rr["dw_read_" + kind][0], rr["dw_store"][0])
        cur = {k: r["expand_store"][0] + r["dw_read_" + k][0] + r["dw_store"][0] for k in ("b64r", "r2b64", "b128r")}
        for kind, b in best.items():
            print(f"    {kind:6s} now {cur[kind]:6d}  best {b[0]:6d} at PW {b[1]} plane pad {b[2]} tile pad {b[3]} "
                  f"(stores {b[4]}, reads {b[5]}, tile {b[6]})")
