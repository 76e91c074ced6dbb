"""Pinhole camera ("PPC") of the shadow-mapping path -- models/camera.py:5-132.

Setup-time 3x3 algebra on the host (one matrix per pose, built once per
dataset); the per-ray work that uses these matrices runs in
``nr_sm_forward``.  Same attribute names as the reference (``camera`` = the
3x3 [a b c] matrix, ``eye_pos``) so code that builds a ``Camera`` and hands it
to ``efficient_sm`` keeps working.
"""
from __future__ import annotations

import math

import numpy as np
import torch

__all__ = ["Camera"]


class Camera:
    def __init__(self, hfov, res):
        """camera.py:6-18: hfov in degrees, res = (w, h)."""
        self.camera = self.initialize_camera_matrix(hfov, res)
        self.res = res
        self._coord_trans = torch.tensor([[1, 0, 0, 0], [0, 0, -1, 0], [0, 1, 0, 0],
                                          [0, 0, 0, 1]], dtype=torch.float32)

    @staticmethod
    def initialize_camera_matrix(hfov, res):
        """camera.py:20-31: columns a = x, b = -y, c = corner ray (fp32 like the
        reference, which builds it from float32 tensors)."""
        w, h = res
        hfovd = torch.tensor(hfov) / torch.tensor(180.0) * math.pi
        a = torch.tensor([1.0, 0.0, 0.0])
        b = torch.tensor([0.0, -1.0, 0.0])
        c = torch.tensor([-w / 2.0, h / 2, -w / (2 * torch.tan(hfovd / 2.0))])
        return torch.stack([a, b, c]).T

    def get_a(self):
        return self.camera[:, 0]

    def get_b(self):
        return self.camera[:, 1]

    def get_c(self):
        return self.camera[:, 2]

    @classmethod
    def from_camera_eyepos(cls, eye_pos, camera):
        """camera.py:42-48."""
        c = cls(30, (400, 400))
        c.res = None
        c.camera = camera
        c.eye_pos = eye_pos
        return c

    @staticmethod
    def c2w_from_lookat(eye_pos, look_at_point, up_guidance=np.array([0, 1, 0], dtype=np.float32)):
        """camera.py:50-67."""
        back = eye_pos - look_at_point
        back = back / np.linalg.norm(back)
        right = np.cross(up_guidance, back)
        right = right / np.linalg.norm(right)
        up = np.cross(back, right)
        m = np.empty((4, 4), dtype=np.float32)
        m[:3, 0], m[:3, 1], m[:3, 2], m[:3, 3] = right, up, back, eye_pos
        m[3, :] = [0, 0, 0, 1]
        return m

    def set_pose_using_blender_matrix(self, c2w, transform_coords=False):
        """camera.py:69-93: eye = c2w[:, 3]; camera = c2w[:, :3] @ camera."""
        if transform_coords:
            raise ValueError("This is not needed anymore. please do not use this flag.")
        self.eye_pos = c2w[:, 3].float()
        self.camera = c2w[:, :3].float() @ self.camera.float()

    def set_camera_matrix(self, eye_pos, lookAtPoint, upGuidance):
        """camera.py:95-119."""
        w, h = self.res
        self.upGuidance = torch.tensor(upGuidance)
        self.lookAtPoint = torch.tensor(lookAtPoint)
        self.eye_pos = torch.tensor(eye_pos)
        newvd = (self.lookAtPoint - self.eye_pos) / torch.linalg.norm(self.lookAtPoint - self.eye_pos)
        cr = torch.cross(newvd, self.upGuidance, dim=-1)
        newa = cr / torch.linalg.norm(cr)
        cr = torch.cross(newvd, newa, dim=-1)
        newb = cr / torch.linalg.norm(cr)
        cr = torch.cross(self.camera[:, 0], self.camera[:, 1], dim=-1)
        focal = torch.dot(cr / torch.linalg.norm(cr), self.camera[:, 2])
        newc = newvd * focal - newa * w / 2.0 - newb * h / 2.0
        self.camera = torch.stack([newa, newb, newc]).T

    def get_transformation_to(self, to_camera, device="cpu"):
        """camera.py:121-132: (R, Q) with R = M_to^-1 M, Q = M_to^-1 (O - O_to)."""
        ml_inv = torch.inverse(to_camera.camera).to(device)
        q = ml_inv @ (self.eye_pos.to(device) - to_camera.eye_pos.to(device))
        return ml_inv @ self.camera.to(device), q
