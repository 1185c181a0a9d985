"""Data-parallel training entry (one rank per GPU under torch.distributed.run; see scripts/launch_dp.sh)."""
from __future__ import annotations

import argparse


def main(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument("--preset", default="a2c_dp8")
    p.add_argument("overrides", nargs="*", help="key=value config overrides")
    a = p.parse_args(argv)
    from ..api import train
    from ..config import TrainConfig, preset
    import dataclasses
    types = {f.name: f.type for f in dataclasses.fields(TrainConfig)}
    kw = {}
    for kv in a.overrides:
        k, v = kv.split("=", 1)
        t = types.get(k, "str")
        if v.lower() in ("none", "null"):
            kw[k] = None
        elif "bool" in str(t):
            kw[k] = v.lower() in ("1", "true", "yes")
        elif "int" in str(t):
            kw[k] = int(v)
        elif "float" in str(t):
            kw[k] = float(v)
        else:
            kw[k] = v
    res = train(preset(a.preset, **kw))
    print("done: %d iterations, %.1f env-steps/s (whole job)" % (res.iterations, res.env_steps_per_sec))


if __name__ == "__main__":
    main()
