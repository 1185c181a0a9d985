"""Configuration surface: one typed config, validated; kernel selection in ``EngineOpts``, not in
hidden process-global environment variables."""
import os
import re

import pytest

from actor_critic_algs_on_tensorflow_amd.config import CHOICES, EngineOpts, TrainConfig, preset

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# every environment variable of this project the package (Python and native code) reads: tooling / A-B switches
# only (alternative library build, reference-op routing, GEMM autotuning and its plans file) -- none selects a kernel
ALLOWED_ENV = {"ACAMD_LIB", "ACAMD_FORCE_REFERENCE", "ACAMD_GEMM_TUNE", "ACAMD_GEMM_PLANS"}


def _env_reads():
    pat = re.compile(r"""(?:environ(?:\.get)?\(?\[?|getenv\()\s*["'](ACA[A-Z0-9_]*)["']""")
    found = set()
    for base in ("actor_critic_algs_on_tensorflow_amd", "csrc"):
        for dirpath, _, files in os.walk(os.path.join(ROOT, base)):
            for f in files:
                if f.endswith((".py", ".cpp", ".h", ".hip")):
                    with open(os.path.join(dirpath, f)) as fh:
                        found |= set(pat.findall(fh.read()))
    return found


def test_package_reads_at_most_ten_project_env_vars():
    found = _env_reads()
    assert found <= ALLOWED_ENV, sorted(found - ALLOWED_ENV)
    assert len(ALLOWED_ENV) <= 10


def test_choice_fields_are_validated():
    for name, allowed in CHOICES.items():
        assert getattr(TrainConfig(), name) in allowed, name
        with pytest.raises(ValueError, match=name):
            TrainConfig(**{name: "no-such-value"})


def test_linear_lr_decay_rejected_with_kl_adaptive_lr():
    with pytest.raises(ValueError, match="kl_adaptive_lr"):
        preset("basic_ac", lr_schedule="linear")
    preset("basic_ac", lr_schedule="linear", kl_adaptive_lr=False)


def test_engine_opts_typed_and_round_trips():
    c = preset("pong_a2c", engine_opts=dict(fused_step=False, nhwc_planes=128))
    assert isinstance(c.engine_opts, EngineOpts) and not c.engine_opts.fused_step and c.engine_opts.nhwc_planes == 128
    d = c.to_dict()
    assert TrainConfig(**d) == c
    with pytest.raises(TypeError):
        EngineOpts(no_such_knob=1)


def test_engine_opts_field_list_is_pinned():
    """Every EngineOpts switch is the default path of a BASELINE config or a test oracle; variants that measured
    slower were deleted with their kernels (fused_fc, per-sample conv1_fold, trunk_bwd_v2, mlp_prefetch, conv1_wgrad
    v1, conv_wgrad_nhwc, cnn_trunk_fwd_u8). A new knob must be added here on purpose."""
    import dataclasses
    names = [f.name for f in dataclasses.fields(EngineOpts)]
    assert names == ["fused_step", "trunk_rows_max_b", "fused_env_split", "adam_step_offsets", "frag_weights",
                     "fc_max_planes", "fc_frag_big", "fc_frag", "a2c_head", "a2c_head_env", "fused_head", "grouped",
                     "det_wgrad", "fused_bwd", "mb_index", "ppo_head", "fc_bwd", "large_batch_min_b",
                     "trunk_bwd_persist", "wgrad_planes", "conv1_v2_planes", "nhwc_planes"]
    assert len(names) <= 25
