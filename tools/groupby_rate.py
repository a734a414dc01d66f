"""Config 5 through XFL's pandas calls (bench.measure_dropin_histogram), plus a
cProfile of one 64-feature pass: where the host time of the per-feature
groupby(col)['xfl_grad_hess'].agg({'count', 'sum'}) goes.
    python tools/groupby_rate.py [--features 64] [--profile]"""
import argparse
import cProfile
import io
import json
import os
import pstats
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--features", type=int, default=64)
    ap.add_argument("--profile", action="store_true")
    args = ap.parse_args()
    import torch
    torch.cuda.init()
    import bench
    from xfl_amd.paillier import PaillierContext
    p, q, n, h = bench.make_key(2048, seed=2024)
    ctx = PaillierContext().init(p, q, djn_h_pow_n=h)
    t0 = time.time()
    rec = bench.measure_dropin_histogram(ctx, nfeat=args.features)
    rec["total_s"] = time.time() - t0
    print(json.dumps(rec), flush=True)
    if args.profile:
        import pandas as pd
        from xfl_amd.paillier import Paillier
        from xfl_amd.paillier_acceleration import embed
        g, hh, values = bench.xgb_inputs(100_000, args.features)
        enc = Paillier.encrypt(ctx, embed([g, hh], interval=1 << 128, precision=64), precision=0)
        gh = Paillier.ciphertext_from(ctx.to_public(), Paillier.serialize(enc, compression=False), compression=False)
        data = pd.concat([pd.DataFrame(gh, columns=['xfl_grad_hess']), values], axis=1)
        cols = list(values.columns)
        [data.groupby([c])['xfl_grad_hess'].agg({'count', 'sum'}) for c in cols[:2]]
        torch.cuda.synchronize()
        pr = cProfile.Profile()
        pr.enable()
        res = [data.groupby([c])['xfl_grad_hess'].agg({'count', 'sum'}) for c in cols]
        torch.cuda.synchronize()
        pr.disable()
        s = io.StringIO()
        pstats.Stats(pr, stream=s).sort_stats("cumulative").print_stats(45)
        print(s.getvalue(), file=sys.stderr)
        del res


if __name__ == "__main__":
    main()
