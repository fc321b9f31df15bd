import torch
import torch.nn.functional as F


def look(vertices, viewpoints, direction=None, up=None):
    """Camera looking along `direction` (reference look.py:5-42); cross products with dim=-1 (see
    look_at.py)."""
    assert vertices.ndim == 3
    device = vertices.device

    def vec(t, default):
        t = default if t is None else t
        if not torch.is_tensor(t):
            t = torch.as_tensor(t, dtype=torch.float32)
        t = t.to(device)
        return t[None, :] if t.ndim == 1 else t

    direction = vec(direction, [0, 0, 1])
    up = vec(up, [0, 1, 0])
    viewpoints = vec(viewpoints, None)

    z_axis = F.normalize(direction)
    x_axis = F.normalize(torch.cross(up.expand_as(z_axis), z_axis, dim=-1))
    y_axis = F.normalize(torch.cross(z_axis, x_axis, dim=-1))
    r = torch.cat((x_axis[:, None, :], y_axis[:, None, :], z_axis[:, None, :]), 1)
    if r.shape[0] != vertices.shape[0]:
        r = r.expand(vertices.shape)
    if vertices.shape != viewpoints.shape:
        viewpoints = viewpoints[:, None, :].expand(vertices.shape)
    return torch.matmul(vertices - viewpoints, r.transpose(1, 0))
