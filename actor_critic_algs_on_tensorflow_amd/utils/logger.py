"""Training-statistics logger with the reference's text-file format, plus a JSONL metrics sidecar.

Parity: ``Basic_AC/util.py:50-106`` / ``A3C/util.py:55-111``.
  * header ``step avg_rew ev_before ev_after act_loss crit_loss kl_dist avg_ent``
  * rows ``'%d %.4f %.4f  %.4f %.4f  %.4f %.4f %.4f'`` (the double spaces are part of the format)
  * the stdout report block printed when ``print_tog`` is true.

Reference bug #8: ``flush`` sets ``last_write = + n`` instead of ``+=``, so step indices are
wrong from the third flush on, and ``__del__`` closes without flushing. By default this logger writes correct
indices and flushes on close; ``legacy_step_index=True`` reproduces the reference numbering bit-for-bit.
"""
from __future__ import annotations

import json
import os
import time

HEADER = "step avg_rew ev_before ev_after act_loss crit_loss kl_dist avg_ent\n"
ROW_FMT = "%d %.4f %.4f  %.4f %.4f  %.4f %.4f %.4f\n"


def format_report(t, avg_rew, ev_before, ev_after, act_loss, circ_loss, act_lr, kl_dist, avg_ent, worker_id):
    """The stdout block of ``Basic_AC/util.py:64-75``."""
    return (
        "\nIteration %d\n" % t
        + "EpRewMean %.4f \n" % avg_rew
        + "EV Before %f\n" % ev_before
        + "EV After %f\n" % ev_after
        + "Act losses %.4f  \n" % act_loss
        + "Critic loss  %.4f\n" % circ_loss
        + "Actor lr %f\n" % act_lr
        + "KL dist %.4f\n" % kl_dist
        + "Avg Ent %.4f\n" % avg_ent
        + "Performed by worker %d" % worker_id
    )


class Logger:
    """Buffers per-iteration stats; ``flush()`` appends rows to ``logfile``.

    ``metrics_path`` (optional) receives one JSON object per ``log_metrics`` call (env-steps/sec, phase
    timers, per-rank stats) -- a sidecar that the reference does not have.
    """

    def __init__(self, logfile, legacy_step_index=False, metrics_path=None, quiet=False):
        self.logfile = logfile
        dir_name = os.path.dirname(logfile)
        if dir_name and not os.path.exists(dir_name):
            os.makedirs(dir_name, exist_ok=True)
        self.f = open(logfile, "w")
        self.last_write = 0
        self.legacy_step_index = legacy_step_index
        self.quiet = quiet
        self.f.write(HEADER)
        self._metrics = open(metrics_path, "a") if metrics_path else None
        self._reset()

    def __call__(self, t, act_loss, circ_loss, kl_dist, avg_rew, print_tog, act_lr, avg_ent, worker_id=0,
                 ev_before=-1, ev_after=-1):
        if print_tog and not self.quiet:
            print(format_report(t, avg_rew, ev_before, ev_after, act_loss, circ_loss, act_lr, kl_dist, avg_ent,
                                worker_id), flush=True)
        self.act_loss.append(float(act_loss))
        self.circ_loss.append(float(circ_loss))
        self.rews.append(float(avg_rew))
        self.ev_before.append(float(ev_before))
        self.ev_after.append(float(ev_after))
        self.kl_dist.append(float(kl_dist))
        self.ents.append(float(avg_ent))

    def _reset(self):
        self.act_loss, self.circ_loss, self.rews = [], [], []
        self.ev_before, self.ev_after, self.kl_dist, self.ents = [], [], [], []

    def flush(self):
        n = len(self.rews)
        for i in range(n):
            self.f.write(ROW_FMT % (i + self.last_write, self.rews[i], self.ev_before[i], self.ev_after[i],
                                    self.act_loss[i], self.circ_loss[i], self.kl_dist[i], self.ents[i]))
        self.f.flush()
        self._reset()
        if self.legacy_step_index:
            self.last_write = +n  # reference behaviour (util.py:106)
        else:
            self.last_write += n

    def log_metrics(self, **kv):
        if self._metrics is not None:
            kv.setdefault("time", time.time())
            self._metrics.write(json.dumps(kv) + "\n")
            self._metrics.flush()

    def close(self):
        if self.f is not None and not self.f.closed:
            if not self.legacy_step_index:
                self.flush()
            self.f.close()
        if self._metrics is not None and not self._metrics.closed:
            self._metrics.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
