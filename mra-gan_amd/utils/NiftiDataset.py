"""Import target for `from utils.NiftiDataset import *` (reference train.py:3-4, test.py:4-5).

The reference's SimpleITK dataset/augmentation module (utils/NiftiDataset.py) is outside this
package's scope: training data reaches `CycleGANModel.set_input` as float32 NCDHW tensors from
the caller's own loader (the reference's train.py uses MONAI transforms, not this module).  With
this package first on sys.path the reference scripts still import; touching any of the old
module's names raises with an explanation instead of failing at import time.
"""

__all__ = []


def __getattr__(name):
    if name.startswith("__"):
        raise AttributeError(name)
    raise NotImplementedError(
        f"utils.NiftiDataset.{name}: the SimpleITK NIfTI dataset/augmentation module is not part of the "
        "MI355X engine; feed float32 [B,C,D,H,W] patches to CycleGANModel.set_input from your own loader "
        "(e.g. the MONAI pipeline in train.py)")
