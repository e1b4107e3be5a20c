"""Load a committed golden fixture back into a Window (test infrastructure)."""
import os

import numpy as np

from ldso_amd import Window

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def make_images(I, w, h):
    """FrameHessian::makeImages level 0 (FrameHessian.cc:68-105) on float32 intensities."""
    N = I.shape[0]
    dI = np.zeros((N, w * h, 3), np.float32)
    for f in range(N):
        img = I[f].astype(np.float32)
        dI[f, :, 0] = img
        idx = np.arange(w, w * (h - 1))
        dx = np.float32(0.5) * (img[idx + 1] - img[idx - 1])
        dy = np.float32(0.5) * (img[idx + w] - img[idx - w])
        dx[np.isnan(dx) | (np.abs(dx) > 255.0)] = 0
        dy[np.isnan(dy) | (np.abs(dy) > 255.0)] = 0
        dI[f, idx, 1] = dx
        dI[f, idx, 2] = dy
    return dI


def load(name):
    z = np.load(os.path.join(GOLDEN, f"{name}.npz"), allow_pickle=False)
    w = Window(n_frames=int(z["n_frames"]), width=int(z["width"]), height=int(z["height"]), calib=z["calib"],
               frames=z["frames"], dI=make_images(z["I"], int(z["width"]), int(z["height"])),
               frame_energy_th=z["frame_energy_th"], point_host=z["point_host"], point_data=z["point_data"],
               point_res_begin=z["point_res_begin"], res_target=z["res_target"], res_state=z["res_state"],
               res_energy=z["res_energy"], res_flags=z["res_flags"])
    w.refresh_frame_terms()
    return w, {k[4:]: z[k] for k in z.files if k.startswith("out_")}, z


NAMES = ["w3_p64", "w5_p160", "w7_p256"]
