"""Host helpers of the public API (reference utils.py:18-72).  The index/mask helpers of the
reference (to_map, MaskForeground, pad_zeros, maximum: utils.py:75-160) have no counterpart here:
their work happens inside the HIP kernels (csrc/nr_raster.hip)."""
import numpy as np
import torch


def make_gif(working_directory, filename):
    """utils.py:10-15: the frames _tmp_*.png of working_directory into an animated GIF (8/100 s per
    frame, looping), then the frames are removed.  PIL's GIF writer stands in for ImageMagick."""
    import glob
    import os
    from PIL import Image
    paths = sorted(glob.glob('%s/_tmp_*.png' % working_directory))
    frames = [Image.open(p).convert('P') for p in paths]
    if frames:
        frames[0].save(filename, save_all=True, append_images=frames[1:], duration=80, loop=0)
    for p in paths:
        os.remove(p)


def to_gpu(data, device=None):
    """utils.py:18-22: move array(s) to a GPU tensor."""
    if isinstance(data, (tuple, list)):
        return [torch.as_tensor(d).cuda(device) for d in data]
    return torch.as_tensor(data).cuda(device)


def imread(filename):
    """utils.py:25-27, PIL-backed (imageio is not part of this image): float32 in [0, 1]."""
    from PIL import Image
    return np.asarray(Image.open(filename), dtype='float32') / 255.


def create_textures(num_faces, texture_size=16, flatten=False):
    """utils.py:30-52: a white texture atlas with one texture_size^2 tile per face."""
    if not flatten:
        tile_width = int((num_faces - 1.) ** 0.5) + 1
        tile_height = int((num_faces - 1.) / tile_width) + 1
    else:
        tile_width, tile_height = 1, num_faces
    textures = np.ones((3, tile_height * texture_size, tile_width * texture_size), 'float32')
    n = np.arange(num_faces)
    col = n % tile_width
    row = n // tile_width
    uv = np.zeros((num_faces, 3, 2), 'float32')
    uv[:, 0, 0] = col * texture_size
    uv[:, 0, 1] = row * texture_size
    uv[:, 1, 0] = col * texture_size
    uv[:, 1, 1] = (row + 1) * texture_size - 1
    uv[:, 2, 0] = (col + 1) * texture_size - 1
    uv[:, 2, 1] = (row + 1) * texture_size - 1
    faces = np.arange(num_faces * 3).reshape((num_faces, 3)).astype('int32')
    return uv.reshape((num_faces * 3, 2)), faces, textures


def get_points_from_angles(distance, elevation, azimuth, degrees=True):
    """utils.py:55-72: camera position on a sphere."""
    if isinstance(distance, (float, int)):
        if degrees:
            elevation = np.radians(elevation)
            azimuth = np.radians(azimuth)
        return (distance * np.cos(elevation) * np.sin(azimuth),
                distance * np.sin(elevation),
                -distance * np.cos(elevation) * np.cos(azimuth))
    if degrees:
        elevation = elevation / 180. * 3.14159265359
        azimuth = azimuth / 180. * 3.14159265359
    return torch.stack([distance * torch.cos(elevation) * torch.sin(azimuth),
                        distance * torch.sin(elevation),
                        -distance * torch.cos(elevation) * torch.cos(azimuth)]).permute(1, 0)
