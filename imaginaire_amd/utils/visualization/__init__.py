from .common import (tensor2im, tensor2label, tensor2flow, tensor2pilimage, Colorize,
                     make_grid, save_image, save_image_grid)  # noqa: F401
