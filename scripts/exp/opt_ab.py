"""Optimiser kernel A/B across builds: runs adam_step / rmsprop_step / opt_multi (PS-style element clip, lr from a
payload slot) for a few steps on seeded inputs and saves every output; with --ref FILE compares bit for bit against
a previous build's file. GPU only."""
import argparse
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
import torch  # noqa: E402

from actor_critic_algs_on_tensorflow_amd.ops.optim import FlatParams, FusedAdam, FusedRMSprop, FusedGroupStep  # noqa


def run():
    dev = "cuda:0"
    g = torch.Generator(device="cpu").manual_seed(7)
    out = {}
    for case in ("adam", "adam_clip", "rms_norm", "multi_ps"):
        ps = [torch.nn.Parameter(torch.randn(n, generator=g).to(dev)) for n in (1000, 4099, 37)]
        flat = FlatParams({"actor": ps[:2], "critic": ps[2:]}, device=dev)
        if case == "multi_ps":
            oa = FusedAdam(flat, "actor", lr=0.05, clip_value=0.1)
            oc = FusedAdam(flat, "critic", lr=1e-3, clip_value=0.1)
            step = FusedGroupStep([oa, oc]).step
            opts = [oa, oc]
        else:
            cls = FusedRMSprop if case == "rms_norm" else FusedAdam
            kw = dict(max_grad_norm=0.5) if case == "rms_norm" else (dict(clip_value=0.05) if case == "adam_clip" else {})
            opts = [cls(flat, "actor", lr=1e-2, **kw), cls(flat, "critic", lr=1e-2, **kw)]
            step = lambda: [o.step() for o in opts]
        for it in range(4):
            flat.grad.copy_(torch.randn(flat.numel, generator=g).to(dev))
            step()
        torch.cuda.synchronize()
        out[case + "_p"] = flat.data.cpu().clone()
        for k, o in enumerate(opts):
            out[f"{case}_v{k}"] = o.v.cpu().clone()
            out[f"{case}_t{k}"] = o.t.cpu().clone()
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--save")
    ap.add_argument("--ref")
    a = ap.parse_args()
    out = run()
    if a.save:
        torch.save(out, a.save)
    if a.ref:
        ref = torch.load(a.ref, weights_only=True)
        bad = [k for k in ref if not torch.equal(ref[k], out[k])]
        for k in bad:
            d = (ref[k].double() - out[k].double()).abs()
            print("DIFF", k, float(d.max()), int((d > 0).sum()))
        print("bitwise equal" if not bad else f"{len(bad)} tensors differ")


if __name__ == "__main__":
    main()
