"""Wavefront OBJ writer (reference save_obj.py:5-47), PIL-backed texture image."""
import os

import numpy as np


def save_obj(filename, vertices, faces, vertices_t=None, faces_t=None, textures=None):
    assert vertices.ndim == 2
    assert faces.ndim == 2
    if textures is not None:
        from PIL import Image
        filename_mtl = filename[:-4] + '.mtl'
        filename_texture = filename[:-4] + '.png'
        material_name = 'material_1'
        textures = textures[:, ::-1, :]
        img = np.clip(np.asarray(textures).transpose((1, 2, 0)) * 255, 0, 255).round().astype(np.uint8)
        Image.fromarray(img).save(filename_texture)
    with open(filename, 'w') as f:
        f.write('# %s\n#\n\n' % os.path.basename(filename))
        if textures is not None:
            f.write('mtllib %s\n\n' % os.path.basename(filename_mtl))
        for v in vertices:
            f.write('v %.8f %.8f %.8f\n' % (v[0], v[1], v[2]))
        f.write('\n')
        if textures is not None:
            vt = np.array(vertices_t, dtype=np.float64, copy=True)
            vt[:, 0] /= (textures.shape[2] - 1)
            vt[:, 1] /= (textures.shape[1] - 1)
            for v in vt.reshape((-1, 2)):
                f.write('vt %.8f %.8f\n' % (v[0], v[1]))
            f.write('\n')
            f.write('usemtl %s\n' % material_name)
            for face, face_t in zip(faces, faces_t):
                f.write('f %d/%d %d/%d %d/%d\n' % (face[0] + 1, face_t[0] + 1, face[1] + 1, face_t[1] + 1,
                                                   face[2] + 1, face_t[2] + 1))
            f.write('\n')
        else:
            for face in faces:
                f.write('f %d %d %d\n' % (face[0] + 1, face[1] + 1, face[2] + 1))
    if textures is not None:
        with open(filename_mtl, 'w') as f:
            f.write('newmtl %s\nmap_Kd %s\n' % (material_name, os.path.basename(filename_texture)))
