"""Drop-in for the reference's test.py: sliding-window inference of one volume with a trained
generator (TestOptions, `--model test`).  The array work runs on the device
(mragan_hip/sliding_window.py); file I/O uses SimpleITK when it is installed (as the reference
does, test.py:42-48, 199-205) and plain `.npy` volumes [x, y, z] otherwise.

    python test.py --image vol.nii --result out.nii --netG resnet_9blocks --name <exp> [--which_epoch latest]
"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from mragan_hip.sliding_window import inference_array  # noqa: E402
from models import create_model  # noqa: E402
from options.test_options import TestOptions  # noqa: E402


def _read(path):
    if path.endswith(".npy"):
        return np.load(path, allow_pickle=False), None
    import SimpleITK as sitk      # the reference's reader; not part of the device path
    img = sitk.ReadImage(path)
    return np.transpose(sitk.GetArrayFromImage(img), (2, 1, 0)).astype(np.float32), img


def _write(path, arr, ref_img):
    if ref_img is None:
        np.save(path, arr)
        return
    import SimpleITK as sitk
    out = sitk.GetImageFromArray(np.transpose(arr, (2, 1, 0)))
    out.SetOrigin(ref_img.GetOrigin())
    out.SetDirection(ref_img.GetDirection())
    out.SetSpacing(ref_img.GetSpacing())
    sitk.WriteImage(out, path)


def inference(model, image_path, result_path, resample, resolution, patch_size_x, patch_size_y, patch_size_z,
              stride_inplane, stride_layer, batch_size=1):
    """test.py:38-207 (resampling to a new resolution is not supported: --resample False)."""
    if resample is True:
        raise NotImplementedError("--resample True needs SimpleITK's BSpline resampler (not part of this engine)")
    image, ref = _read(image_path)
    label = inference_array(model, image, (int(patch_size_x), int(patch_size_y), int(patch_size_z)),
                            int(np.ravel([stride_inplane])[0]), int(np.ravel([stride_layer])[0]))
    _write(result_path, label, ref)
    print("Save evaluate label at {} success".format(result_path))


if __name__ == '__main__':
    opt = TestOptions().parse()
    model = create_model(opt)
    model.setup(opt)
    inference(model, opt.image, opt.result, opt.resample, opt.new_resolution, opt.patch_size[0],
              opt.patch_size[1], opt.patch_size[2], opt.stride_inplane, opt.stride_layer, 1)
