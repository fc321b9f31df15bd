// nr_host.h -- host-side argument validation and Shade construction
// Part of nr_raster.hip (one translation unit); see that file and DESIGN.md.
#pragma once

#pragma clang fp contract(off)

namespace {

int validate_raster(const NrRasterArgs* a, bool need_workspace) {
    if (!a) return fail(NR_ERR_ARGS, "null args");
    if (a->batch_size < 0 || a->num_faces < 0 || a->num_vertices < 0 || a->image_size <= 0)
        return fail(NR_ERR_ARGS, "bad sizes B=%d F=%d V=%d s=%d", a->batch_size, a->num_faces, a->num_vertices,
                    a->image_size);
    const int S = a->anti_aliasing ? 2 * a->image_size : a->image_size;
    if (S > 16384) return fail(NR_ERR_ARGS, "image too large (%d internal pixels per side)", S);
    if (nr_num_channels(a->draw_flags) == 0) return fail(NR_ERR_ARGS, "nothing to draw");
    if (a->batch_size > 0 && a->num_faces > 0 && (!a->vertices || !a->faces || !a->face_records))
        return fail(NR_ERR_ARGS, "null vertices/faces/face_records");
    if (a->batch_size > 0 && !a->face_index) return fail(NR_ERR_ARGS, "null face_index");
    if (a->draw_flags & NR_DRAW_RGB) {
        if (!a->vertices_textures || !a->faces_textures || !a->textures || !a->face_uv)
            return fail(NR_ERR_ARGS, "rgb requested without textures");
        if (a->tex_height <= 0 || a->tex_width <= 0) return fail(NR_ERR_ARGS, "bad texture size");
        if (a->num_lights < 0) return fail(NR_ERR_ARGS, "negative light count");
        if (a->num_lights > 0 && (!a->lights || !a->vertex_normals || !a->face_normals || !a->normal_offsets ||
                                  !a->normal_faces))
            return fail(NR_ERR_ARGS, "lights need lights / face_normals / vertex_normals / normal CSR buffers");
        const long long span = 2 * std::llabs(a->tex_stride_c) +
                               ((long long)a->tex_height * a->tex_width - 1) * std::llabs(a->tex_stride_p) + 1;
        if (span >= (1ll << 31)) return fail(NR_ERR_ARGS, "texture item spans 2^31 elements or more");
    }
    const Geom g = make_geom(a->num_faces, S);
    const size_t need = ws_bbox_bytes(a->batch_size, a->num_faces) + ws_mask_bytes(a->batch_size, g) + ws_order_bytes(a->batch_size, g);
    if (need_workspace && need > 0 && (!a->workspace || a->workspace_bytes < need))
        return fail(NR_ERR_WORKSPACE, "workspace missing or too small");
    return NR_OK;
}

Shade make_shade(const NrRasterArgs* a) {
    Shade sh;
    sh.draw = a->draw_flags;
    sh.C = nr_num_channels(a->draw_flags);
    sh.eps = a->eps;
    sh.tv.tex = a->textures;
    sh.tv.sb = a->tex_stride_b;
    sh.tv.sc = (int)a->tex_stride_c;
    sh.tv.sp = (int)a->tex_stride_p;
    sh.tv.H = a->tex_height;
    sh.tv.W = a->tex_width;
    sh.tv.t4 = reinterpret_cast<const float4*>(a->textures_packed);
    sh.tv.HWp = (a->tex_height * a->tex_width + 3) & ~3;
    sh.face_uv = a->face_uv;
    sh.uv_bstride = a->vt_batch_stride ? (long long)a->num_faces * 8 : 0;
    const bool rgb = (a->draw_flags & NR_DRAW_RGB) != 0;
    sh.nl = rgb ? a->num_lights : 0;
    sh.B = a->batch_size;
    sh.V = a->num_vertices;
    sh.lights = a->lights;
    sh.vnorm = a->vertex_normals;
    sh.fidx = a->faces;
    sh.bg = rgb ? a->backgrounds : nullptr;
    sh.bg_sb = a->bg_stride_b;
    sh.bg_sc = (int)a->bg_stride_c;
    sh.bg_sy = (int)a->bg_stride_y;
    return sh;
}

}  // namespace
