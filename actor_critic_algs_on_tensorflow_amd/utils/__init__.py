"""Host-side utilities: schedules, LR controller, reference-format Logger, Framer, statistics, timers."""
from .framer import Framer, FrameStack
from .logger import Logger
from .schedule import DeviceKLAdaptiveLR, KLAdaptiveLR, LinearSchedule, RegularizerSchedule
from .stats import explained_variance, make_np, ob_feature_augment, var_accounted_for

__all__ = ["Framer", "FrameStack", "Logger", "LinearSchedule", "KLAdaptiveLR", "DeviceKLAdaptiveLR",
           "RegularizerSchedule", "var_accounted_for", "explained_variance", "make_np", "ob_feature_augment"]
