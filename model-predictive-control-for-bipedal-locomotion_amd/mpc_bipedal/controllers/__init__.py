"""Controllers for bipedal locomotion."""

from .zmp_controller import ZMPController

__all__ = ['ZMPController']
