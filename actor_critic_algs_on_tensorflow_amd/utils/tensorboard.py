"""TensorBoard event files without TensorFlow (reference C30 / C15: ``tf.summary.FileWriter`` + ``variable_summaries``).

The reference writes, with ``--tboard``, every iteration's merged summaries -- per trainable variable the scalars
mean / stddev / max / min (``Basic_AC/policies.py:9-18``, attached at ``:83-85`` and ``:146-149``) -- to
``summaries/<outdir-stem>.data`` (``Basic_AC/run_AC.py:201-202,253-255``). This module writes the same file format
TensorFlow does, so TensorBoard reads it:

* a file ``events.out.tfevents.<unix time>.<host>`` of TFRecords: ``uint64 length``, ``uint32 masked CRC32C(length)``,
  the serialized ``Event`` proto, ``uint32 masked CRC32C(data)`` (the masked CRC32C comes from the C++ checkpoint
  codec, ``csrc/tfbundle``);
* first record ``Event{wall_time, file_version: "brain.Event:2"}``, then ``Event{wall_time, step, summary}`` with
  ``Summary{value: [{tag, simple_value}]}``.

Per-variable statistics are computed on the device by one native reduction launch over the flat parameter slab
(``param_stats`` in ``ops/stats.py``). Tag names follow TF1 scoping as the reference graph produces
them: ``<Scope>/var_<i>summaries/mean`` and ``<Scope>/stddev[_k]/{stddev,max,min}`` ([TF1-semantics]: the second
``tf.variable_scope('stddev')`` of a graph opens the uniquified name scope ``stddev_1``, and so on).
"""
from __future__ import annotations

import os
import socket
import struct
import time


def _varint(n):
    out = bytearray()
    n &= (1 << 64) - 1
    while True:
        b = n & 0x7F
        n >>= 7
        if n:
            out.append(b | 0x80)
        else:
            out.append(b)
            return bytes(out)


def _key(field, wire):
    return _varint((field << 3) | wire)


def _bytes_field(field, data):
    return _key(field, 2) + _varint(len(data)) + data


def encode_summary(values):
    """``values``: iterable of (tag, float) -> serialized ``Summary``."""
    out = b""
    for tag, v in values:
        val = _bytes_field(1, tag.encode()) + _key(2, 5) + struct.pack("<f", float(v))
        out += _bytes_field(1, val)
    return out


def encode_event(wall_time, step=None, summary=None, file_version=None):
    out = _key(1, 1) + struct.pack("<d", float(wall_time))
    if step is not None:
        out += _key(2, 0) + _varint(int(step))
    if file_version is not None:
        out += _bytes_field(3, file_version.encode())
    if summary is not None:
        out += _bytes_field(5, summary)
    return out


def _crc(b):
    from ..ckpt import codec
    return codec.masked_crc32c(b)


def frame_record(data):
    head = struct.pack("<Q", len(data))
    return head + struct.pack("<I", _crc(head)) + data + struct.pack("<I", _crc(data))


class SummaryWriter:
    """Minimal ``tf.summary.FileWriter``: scalars (and the reference's per-variable statistics)."""

    def __init__(self, logdir, filename_suffix=""):
        os.makedirs(logdir, exist_ok=True)
        name = "events.out.tfevents.%d.%s%s" % (int(time.time()), socket.gethostname(), filename_suffix)
        self.path = os.path.join(logdir, name)
        self._f = open(self.path, "wb")
        self._f.write(frame_record(encode_event(time.time(), file_version="brain.Event:2")))
        self._f.flush()

    def add_scalars(self, values, step, wall_time=None):
        """``values``: dict tag -> float (one Event, like a merged summary)."""
        summ = encode_summary(values.items())
        self._f.write(frame_record(encode_event(time.time() if wall_time is None else wall_time, step, summ)))

    def add_scalar(self, tag, value, step, wall_time=None):
        self.add_scalars({tag: value}, step, wall_time)

    def flush(self):
        self._f.flush()

    def close(self):
        if not self._f.closed:
            self._f.flush()
            self._f.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def variable_summary_tags(scopes):
    """``scopes``: list of (scope, n_vars) in graph-creation order -> per scope the list of
    (mean_tag, stddev_tag, max_tag, min_tag) for its variables (TF1 name-scope uniquification, see module doc)."""
    out = []
    for scope, n in scopes:
        tags = []
        for i in range(n):
            sd = "stddev" if i == 0 else "stddev_%d" % i
            tags.append(("%s/var_%dsummaries/mean" % (scope, i), "%s/%s/stddev" % (scope, sd),
                         "%s/%s/max" % (scope, sd), "%s/%s/min" % (scope, sd)))
        out.append(tags)
    return out


def summaries_dir(outdir, root="summaries"):
    """The reference's event directory: ``summaries/<outdir up to the first '.'>.data`` (``Basic_AC/run_AC.py:202``)."""
    return os.path.join(root, str(outdir).split(".")[0] + ".data")


def reference_summary_scopes(actor, critic):
    """The variable lists the reference attaches ``variable_summaries`` to, in graph order.

    ``Basic_AC/run_AC.py:197-198`` builds the Critic before the Actor, and both call ``adam.compute_gradients(loss)``
    without a ``var_list`` (``Basic_AC/policies.py:80,146``), i.e. over EVERY trainable variable that exists at that
    point: the Critic summarises its own 8 variables (``third_layer`` included although ``value`` reads
    ``second_layer``), the Actor summarises the Critic's 8 followed by its own (kernel/bias of the 4 dense layers, then
    the continuous ``log_std``)."""
    crit = []
    for n in ("first_layer", "second_layer", "third_layer", "value"):
        layer = getattr(critic, n, None)
        if layer is not None:
            crit += [layer.kernel, layer.bias]
    act = []
    for n in ("first_layer", "second_layer", "third_layer", "logits" if actor.discrete else "mu_layer"):
        layer = getattr(actor, n, None)
        if layer is not None:
            act += [layer.kernel, layer.bias]
    if not actor.discrete and getattr(actor, "log_std", None) is not None:
        act.append(actor.log_std)
    return [("Critic", crit), ("Actor", crit + act)]


class VariableSummaries:
    """Per-variable mean / stddev / max / min of scoped variable lists, written as one merged Event.

    When every variable lives in one :class:`..ops.optim.FlatParams` slab the statistics come from ONE device
    reduction launch and ONE device->host copy (``ops/stats.py``); otherwise (the CPU parity trainer) per tensor."""

    def __init__(self, writer, scopes, flat=None):
        self.writer = writer
        self.tags = [t for per in variable_summary_tags([(s, len(v)) for s, v in scopes]) for t in per]
        uniq, self.slot, seen = [], [], {}
        for _, vs in scopes:
            for v in vs:
                if id(v) not in seen:
                    seen[id(v)] = len(uniq)
                    uniq.append(v)
                self.slot.append(seen[id(v)])
        self.uniq = uniq
        self.flat, self.segs = None, None
        if flat is not None and all(id(v) in {id(p) for p in flat.params} for v in uniq):
            from ..ops.stats import param_segments
            self.flat = flat
            self.segs = param_segments(flat, uniq)

    def values(self):
        """-> dict tag -> float."""
        if self.flat is not None:
            from ..ops.stats import seg_stats
            st = seg_stats(self.flat.data, self.segs).cpu().tolist()
        else:
            st = []
            for v in self.uniq:
                x = v.detach().double().reshape(-1)
                st.append([x.mean().item(), x.var(unbiased=False).sqrt().item(), x.max().item(), x.min().item()])
        out = {}
        for tags, k in zip(self.tags, self.slot):
            for tag, val in zip(tags, st[k]):
                out[tag] = val
        return out

    def write(self, step, extra=None):
        vals = self.values()
        if extra:
            vals.update(extra)
        self.writer.add_scalars(vals, step)
        return vals

    def close(self):
        self.writer.close()


# ------------------------------------------------------------------------------------------------ reader (tests)
def _read_varint(b, i):
    shift = n = 0
    while True:
        c = b[i]
        i += 1
        n |= (c & 0x7F) << shift
        if c < 0x80:
            return n, i
        shift += 7


def _parse_fields(b):
    i, out = 0, []
    while i < len(b):
        k, i = _read_varint(b, i)
        f, w = k >> 3, k & 7
        if w == 0:
            v, i = _read_varint(b, i)
        elif w == 1:
            v = b[i:i + 8]
            i += 8
        elif w == 5:
            v = b[i:i + 4]
            i += 4
        elif w == 2:
            n, i = _read_varint(b, i)
            v = b[i:i + n]
            i += n
        else:
            raise ValueError("unsupported wire type %d" % w)
        out.append((f, w, v))
    return out


def read_events(path):
    """-> list of dicts {wall_time, step, file_version?, scalars: {tag: value}}; verifies both CRCs per record."""
    data = open(path, "rb").read()
    i, events = 0, []
    while i < len(data):
        head = data[i:i + 8]
        (n,) = struct.unpack("<Q", head)
        (hc,) = struct.unpack("<I", data[i + 8:i + 12])
        if hc != _crc(head):
            raise ValueError("length CRC mismatch at byte %d" % i)
        rec = data[i + 12:i + 12 + n]
        (dc,) = struct.unpack("<I", data[i + 12 + n:i + 16 + n])
        if dc != _crc(rec):
            raise ValueError("data CRC mismatch at byte %d" % i)
        i += 16 + n
        ev = {"scalars": {}}
        for f, w, v in _parse_fields(rec):
            if f == 1:
                ev["wall_time"] = struct.unpack("<d", v)[0]
            elif f == 2:
                ev["step"] = v
            elif f == 3:
                ev["file_version"] = v.decode()
            elif f == 5:
                for f2, _, val in _parse_fields(v):
                    if f2 != 1:
                        continue
                    tag, x = None, None
                    for f3, _, v3 in _parse_fields(val):
                        if f3 == 1:
                            tag = v3.decode()
                        elif f3 == 2:
                            x = struct.unpack("<f", v3)[0]
                    ev["scalars"][tag] = x
        events.append(ev)
    return events
