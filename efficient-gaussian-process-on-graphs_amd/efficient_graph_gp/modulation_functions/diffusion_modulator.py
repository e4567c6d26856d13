from grf_amd.api import diffusion_modulator  # (-beta)^l / (2^l l!)

__all__ = ["diffusion_modulator"]
