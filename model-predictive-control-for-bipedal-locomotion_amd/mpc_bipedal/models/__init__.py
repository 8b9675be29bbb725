"""LIPM model and prediction matrices."""

from .lipm_model import LIPMModel, ModelConfig, lipm_matrices, prediction_matrices, toeplitz_column

__all__ = ['LIPMModel', 'ModelConfig', 'lipm_matrices', 'prediction_matrices', 'toeplitz_column']
