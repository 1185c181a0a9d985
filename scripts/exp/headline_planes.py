"""Headline (Pong A2C, 32 envs x 5) learner gradient plane sets: plane counts of each weight gradient and the bytes the
finaliser reads (planes + final segments), from the engine's job table after one update. GPU only."""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
import torch  # noqa: E402

from actor_critic_algs_on_tensorflow_amd import preset  # noqa: E402
from actor_critic_algs_on_tensorflow_amd.algos.trainer import ActorCriticTrainer  # noqa: E402


def main():
    tr = ActorCriticTrainer(preset("pong_a2c", device="cuda:0", outdir=None, quiet=True, stdout_freq=0, save_every=0,
                                   engine_opts=json.loads(sys.argv[1]) if len(sys.argv) > 1 else {}))
    tr.step()
    torch.cuda.synchronize()
    eng = tr.engine
    out = {"wsplits": dict(eng._wsplits), "cur_planes": dict(eng._cur_planes)}
    for key, (words, mx) in eng._fin_words.items():
        w = words.cpu()
        plane_bytes = int(sum(int(r[2]) * int(r[4]) * 4 for r in w if int(r[1])))
        final_bytes = int(sum(int(r[2]) * 4 for r in w if not int(r[1])))
        out[str(key[:3])] = {"jobs": int(w.shape[0]), "plane_read_MB": round(plane_bytes / 1e6, 2),
                             "final_read_MB": round(final_bytes / 1e6, 2), "largest_job": int(mx)}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
