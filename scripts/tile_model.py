#!/usr/bin/env python3
"""Work model of the fused kernel's tile shapes on one MI355X (no GPU needed).

For an nx x ny x nz sub-domain and depth T it prints, per tile shape (ROWS x WAVES, the
workgroups a CU holds), the computed cell-levels per useful update (x yield 64-2T of 64 lanes,
y yield of the waves' rows inside each level's cone, the partial edge tiles) and the sched-2
schedule's makespan (rounds x (planes per chunk + 2T pipeline fill) x cells per CU and iteration),
i.e. the
VALU issue time per pass up to a constant -- fused.hpp FusedLaunch::run's own chunk choice.

  python scripts/tile_model.py --n 512 512 512 --T 3

The folded last strip (4x12f, fused.hpp FCfg::FOLD) is listed where it applies (e.g. L=256).
"""
import argparse


def model(nx, ny, nz, T, rows, waves, wg_per_cu, cus=256, oy=0, fold=False):
    rt = rows * waves
    ystep = (rt - 2 * T) & ~3
    xstep = 64 - 2 * T
    ybase = -((oy - T) % 4)
    ntx = -(-nx // xstep)
    nty = (ny - ybase + ystep - 1) // ystep
    ntiles = ntx * nty
    # folded last x strip (fused.hpp FCfg::FOLD): its tiles run two per wave when the strip
    # holds <= 32 - 2T outputs
    folded = fold and ntx >= 2 and nx - (ntx - 1) * xstep <= 32 - 2 * T
    if folded:
        ntiles = (ntx - 1) * nty + (nty + 1) // 2
    # rows computed per level l (waves whose rows touch [l+1, need_hi(l)]): k_fused's skip rule
    comp = 0
    for l in range(T):
        hi = 2 * T + ystep - 2 - l
        comp += sum(rows for w in range(waves) if not (w * rows > hi or w * rows + rows - 1 < l + 1))
    useful_rows = T * ystep
    y_yield = useful_rows / comp
    x_yield = xstep / 64
    cover = (nx * ny) / (((ntx - 1) * xstep + (xstep / 2 if folded else xstep)) * nty * ystep)
    per_useful = 1 / (x_yield * y_yield * cover)
    slots = wg_per_cu * cus
    M = max(1, slots // 8)
    best = None
    for nch in range(1, max(1, nz // 2) + 1):
        per = -(-(ntiles * nch) // 8)
        rounds = -(-per // M)
        cost = rounds * (-(-nz // nch) + 2 * T)
        if best is None or cost < best[0]:
            best = (cost, nch, rounds)
    cost, nch, rounds = best
    # VALU time per pass ~ makespan x cells a CU computes per pipeline iteration (VALU-bound CU)
    t = cost * rt * wg_per_cu
    return dict(tile=f"{rows}x{waves}" + ("f" if folded else ""), wg_per_cu=wg_per_cu,
                ntiles=ntiles, ystep=ystep,
                x_yield=round(x_yield, 3), y_yield=round(y_yield, 3), cover=round(cover, 3),
                levels_per_useful=round(per_useful, 3), nch=nch, rounds=rounds,
                busy_cus=round(min(1.0, ntiles * nch / (rounds * slots)), 3), makespan=cost,
                time_units=t)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, nargs=3, default=[512, 512, 512])
    ap.add_argument("--T", type=int, default=3)
    a = ap.parse_args()
    # (rows, waves, workgroups per CU as the register / LDS budget allows, fp32)
    shapes = [(4, 8, 2), (4, 12, 1), (4, 16, 1), (8, 4, 2), (4, 6, 2)]
    rows = [model(*a.n, a.T, r, w, k) for r, w, k in shapes]
    f = model(*a.n, a.T, 4, 12, 1, fold=True)
    if f["tile"].endswith("f"):
        rows.append(f)
    base = next(r["time_units"] for r in rows if r["tile"] == "4x12")
    for r in rows:
        r["rel_time"] = round(r["time_units"] / base, 3)
        print(r)


if __name__ == "__main__":
    main()
