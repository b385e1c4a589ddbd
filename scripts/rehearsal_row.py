#!/usr/bin/env python3
"""One summary block of a multi-rank bench.py JSON line: the headline, the chosen data path,
the link probe's summary and the data-path tuning table (timed, or skipped and why)."""
import json
import sys


def main(path):
    d = json.loads([l for l in open(path) if l.startswith("{")][-1])
    c = d.get("config", {})
    print(f"N={d['n_gpus']} status={d.get('status')} MLUPS={d['value']} ms/step={d['ms_per_step']} "
          f"{c.get('parallelism')} golden={d.get('check', {}).get('golden_ok')} "
          f"tuning_s={d.get('tuning_s')} wall_s={d.get('wall_s')}")
    lp = d.get("link_probe")
    if lp:
        print(f"  link_probe ({lp.get('probe_s')} s, rccl: {str(lp.get('rccl'))[:90]})")
        for k, v in lp.get("summary", {}).items():
            print(f"    {k}: {v}")
    for r in d.get("data_path_tuning") or []:
        what = (f"{r.get('ms_per_step')} ms/step" if r.get("ok") else
                f"skipped: {r.get('skipped')}" if r.get("skipped") else "failed")
        print(f"  {r['dims']} fuse {r['fuse']} {r.get('overlap_req')} "
              f"{r.get('transport_req') or r.get('transport') or ''}: {what}"
              f"  model {r.get('model_ms_per_step')}  comp {r.get('model_comp_ms_per_step')}")


if __name__ == "__main__":
    main(sys.argv[1])
