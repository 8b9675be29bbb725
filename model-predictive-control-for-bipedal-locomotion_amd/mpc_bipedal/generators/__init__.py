"""Generators for footsteps and CoP bounds (the solver's input producer)."""

from .footstep_generator import Contact, generate_footsteps
from .cop_generator import CoPGenerator, State, cop_params, generate_cop_batch
from .speed_generation import SpeedTrajectoryGenerator

__all__ = ['Contact', 'generate_footsteps', 'CoPGenerator', 'State', 'SpeedTrajectoryGenerator',
           'cop_params', 'generate_cop_batch']
