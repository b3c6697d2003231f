"""``fluid.contrib.sparsity`` (reference: python/paddle/fluid/contrib/sparsity): the ASP n:m
structured-sparsity tools of ``paddle.incubate.asp``."""
from ....incubate.asp import *  # noqa: F401,F403
from ....incubate.asp import (CheckMethod, MaskAlgo, calculate_density, check_mask_1d, check_mask_2d,  # noqa: F401
                              check_sparsity, create_mask, decorate, get_mask_1d, get_mask_2d_best,
                              get_mask_2d_greedy, prune_model, set_excluded_layers, reset_excluded_layers)
from ....incubate import asp  # noqa: F401
