"""TF-free parts of the reference's ``code/input_pipelines/utils.py`` that the hot path uses."""
import numpy as np


def from_0_1_to_m1_1(images):
    """[0, 1) -> [-1, 1): (x - 0.5) / 0.5 (input_pipelines/utils.py:96-112)."""
    mean = 0.5
    return (np.asarray(images, dtype=np.float32) - mean) / mean


def get_temp_Nb(runconfig, Nb):
    """Per-tower (per-rank) batch: Nb / num_towers, which must divide (utils.py:118-125)."""
    if getattr(runconfig, 'train_distribute', None):
        div, mod = divmod(Nb, runconfig.train_distribute.num_towers)
        assert not mod, 'for now Nb must be divisible by the number of available GPUs.'
        return div
    return Nb
