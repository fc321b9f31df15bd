"""Wavefront OBJ/MTL loader with texture atlas (reference load_obj.py:7-166), PIL-backed.

The atlas is built in material order: image materials are flipped vertically and their uv scaled
to pixels (load_obj.py:70-82); colour-only materials become 2x2 patches with three synthetic uv
vertices (load_obj.py:84-94); atlas pieces are stacked along H, padded with zeros in W."""
import os

import numpy as np


def _read_image(path):
    from PIL import Image
    return np.asarray(Image.open(path))


def load_mtl(filename_mtl):
    materials = {}
    name = ''
    with open(filename_mtl) as f:
        for line in f:
            tok = line.split()
            if not tok:
                continue
            if tok[0] == 'newmtl':
                name = tok[1]
                materials[name] = {}
            elif tok[0] == 'map_Kd':
                materials[name]['texture_filename'] = tok[1]
            elif tok[0] == 'Kd':
                materials[name]['color'] = np.array(list(map(float, tok[1:4])))
    return materials


def _face_corner(token, slot):
    parts = token.split('/')
    if slot == 0:
        return int(parts[0])
    return int(parts[1]) if '/' in token else 0


def load_textures_func(filename_obj, filename_mtl):
    uv = []
    faces = []
    material_names = []
    material = ''
    with open(filename_obj) as f:
        lines = f.readlines()
    for line in lines:
        tok = line.split()
        if tok and tok[0] == 'vt':
            uv.append([float(v) for v in tok[1:3]])
    uv = np.vstack(uv).astype('float32')
    for line in lines:
        tok = line.split()
        if not tok:
            continue
        if tok[0] == 'f':
            vs = tok[1:]
            v0 = _face_corner(vs[0], 1)
            for i in range(len(vs) - 2):
                faces.append((v0, _face_corner(vs[i + 1], 1), _face_corner(vs[i + 2], 1)))
                material_names.append(material)
        elif tok[0] == 'usemtl':
            material = tok[1]
    faces = np.vstack(faces).astype('int32') - 1
    material_names = np.array(material_names)

    materials = load_mtl(filename_mtl)
    pos = 0
    textures = np.zeros((3, 0, 0), 'float32')
    for name, mat in materials.items():
        if 'texture_filename' in mat:
            tex = _read_image(os.path.join(os.path.dirname(filename_mtl), mat['texture_filename']))
            tex = (tex.astype('float32') / 255.).transpose((2, 0, 1))[:, ::-1, ::1]
            idx = np.unique(faces[material_names == name].flatten())
            uv[idx, 0] *= tex.shape[2] - 1
            uv[idx, 1] *= tex.shape[1] - 1
            uv[idx, 1] += pos
        else:
            tex = np.ones((3, 2, 2), 'float32') * np.array(mat['color'])[:, None, None]
            uv = np.concatenate((uv, np.array([[0, pos], [0, pos + 1], [1, pos + 1]], 'float32')), axis=0)
            faces[material_names == name] = np.array([uv.shape[0] - 3, uv.shape[0] - 2, uv.shape[0] - 1])
        pos += tex.shape[1]
        if textures.shape[2] < tex.shape[2]:
            textures = np.concatenate(
                (textures, np.zeros((3, textures.shape[1], tex.shape[2] - textures.shape[2]))), axis=2)
        elif tex.shape[2] < textures.shape[2]:
            tex = np.concatenate((tex, np.zeros((3, tex.shape[1], textures.shape[2] - tex.shape[2]))), axis=2)
        textures = np.concatenate((textures, tex), axis=1).astype('float32')
    return uv, faces, textures


def load_obj(filename_obj, normalization=True, load_textures=False):
    """Vertices (`v`) and fan-triangulated faces (`f`), optionally textures; normalised into a
    centred cube of side 2 (load_obj.py:113-166)."""
    with open(filename_obj) as f:
        lines = f.readlines()
    vertices = np.vstack([[float(v) for v in l.split()[1:4]] for l in lines
                          if l.split() and l.split()[0] == 'v']).astype('float32')
    faces = []
    for l in lines:
        tok = l.split()
        if tok and tok[0] == 'f':
            vs = tok[1:]
            v0 = _face_corner(vs[0], 0)
            for i in range(len(vs) - 2):
                faces.append((v0, _face_corner(vs[i + 1], 0), _face_corner(vs[i + 2], 0)))
    faces = np.vstack(faces).astype('int32') - 1

    textures = None
    if load_textures:
        for l in lines:
            if l.startswith('mtllib'):
                mtl = os.path.join(os.path.dirname(filename_obj), l.split()[1])
                vertices_t, faces_t, textures = load_textures_func(filename_obj, mtl)
        if textures is None:
            raise Exception('Failed to load textures.')

    if normalization:
        vertices -= vertices.min(0)[None, :]
        vertices /= np.abs(vertices).max()
        vertices *= 2
        vertices -= vertices.max(0)[None, :] / 2

    if load_textures:
        return vertices, faces, vertices_t, faces_t, textures
    return vertices, faces
