"""The relightable render() step on the fused path (SURVEY §8f #1 + #2).

`render` has the signature and outputs of the reference's gaussian_renderer.render
(gaussian_renderer/__init__.py:69-280), and computes them with three ops instead of a
chain of ~60 PyTorch kernels and 6-10 rasterizer calls:

  1. relit_shade.relit_features -- every per-Gaussian channel render() prepares (shaded
     colour, diffuse, specular, depth, normal, alpha; sky colours for sky Gaussians) as
     [P, 16] rows, one HIP pass each way;
  2. diff_gaussian_rasterization.rasterize_channels -- one geometry pass and one
     multi-channel composite of all images (the debug extras add a second 16-channel group);
  3. the reference's image-space post-processing (normal remap, sky masking, normal_ref
     from the depth image), restated in PyTorch.

Each image equals what the reference's separate call produces from the same per-Gaussian
colours (tests/test_gpu_relit.py).  Opt-in: callers import this `render` in place of
gaussian_renderer.render.
"""
import math

import torch


def depths_to_points(view, depthmap):
    """graphics_utils.py:141-156: back-project a depth map through the camera."""
    c2w = view.world_view_transform.T.inverse()
    W, H = view.image_width, view.image_height
    fx = W / (2 * math.tan(view.FoVx / 2.))
    fy = H / (2 * math.tan(view.FoVy / 2.))
    dev = depthmap.device
    intrins = torch.tensor([[fx, 0., W / 2.], [0., fy, H / 2.], [0., 0., 1.0]], device=dev).float()
    gx, gy = torch.meshgrid(torch.arange(W, device=dev).float(), torch.arange(H, device=dev).float(), indexing="xy")
    pts = torch.stack([gx, gy, torch.ones_like(gx)], dim=-1).reshape(-1, 3)
    rays_d = pts @ intrins.inverse().T @ c2w[:3, :3].T
    return depthmap.reshape(-1, 1) * rays_d + c2w[:3, 3]


def depth_to_normal(view, depth):
    """graphics_utils.py:158-169: normals from the depth image by central differences."""
    points = depths_to_points(view, depth).reshape(*depth.shape[1:], 3)
    out = torch.zeros_like(points)
    dx = points[2:, 1:-1] - points[:-2, 1:-1]
    dy = points[1:-1, 2:] - points[1:-1, :-2]
    out[1:-1, 1:-1, :] = torch.nn.functional.normalize(torch.cross(dx, dy, dim=-1), dim=-1)
    return out


def render(viewpoint_camera, pc, envlight, sky_sh, sky_sh_degree, pipe, bg_color, scaling_modifier=1.0, debug=True,
           specular=True, fix_sky=False, normal_view=False):
    """gaussian_renderer/__init__.py:69-280 on the fused path (same arguments, same output
    dictionary: render, viewspace_points, visibility_filter, radii, diffuse_color,
    specular_color, depth, normal, alpha, normal_ref and, with debug, sky_color, roughness,
    metalness, albedo)."""
    import diff_gaussian_rasterization as dgr
    import relit_shade

    screenspace_points = torch.zeros_like(pc.get_xyz, dtype=pc.get_xyz.dtype, requires_grad=True) + 0
    try:
        screenspace_points.retain_grad()
    except Exception:
        pass
    tanfovx = math.tan(viewpoint_camera.FoVx * 0.5)
    tanfovy = math.tan(viewpoint_camera.FoVy * 0.5)
    settings = dgr.GaussianRasterizationSettings(
        image_height=int(viewpoint_camera.image_height), image_width=int(viewpoint_camera.image_width),
        tanfovx=tanfovx, tanfovy=tanfovy, bg=bg_color, scale_modifier=scaling_modifier,
        viewmatrix=viewpoint_camera.world_view_transform, projmatrix=viewpoint_camera.full_proj_transform,
        sh_degree=-1, campos=viewpoint_camera.camera_center, prefiltered=False)

    means3D = pc.get_xyz
    opacity = pc.get_opacity
    empty = torch.Tensor([])
    scales = rotations = cov3D_precomp = empty
    if pipe.compute_cov3D_python:
        cov3D_precomp = pc.get_covariance(scaling_modifier)
    else:
        scales = pc.get_scaling
        rotations = pc.get_rotation
    dev = means3D.device
    sky_mask = viewpoint_camera.sky_mask.to(dev).squeeze()
    is_sky = pc.get_is_sky.squeeze()

    feat = relit_shade.relit_features(means3D, pc.get_rotation, pc.get_scaling, is_sky, pc.get_albedo,
                                      pc.get_roughness, pc.get_metalness, envlight, viewpoint_camera.camera_center,
                                      viewpoint_camera.world_view_transform, sky_sh, sky_sh_degree, specular, fix_sky)
    bg = bg_color.reshape(-1).float()
    # A value repeated over three channels (depth, alpha, roughness, metalness) is one
    # composite channel when the background is grey; otherwise three.
    grey = bool((bg == bg[0]).all())
    zero3 = torch.zeros(3, device=dev)
    # (name, columns [P, k], background [k]); alpha is rendered with a black background
    chans = [("render", feat[:, 0:3], bg), ("diffuse_color", feat[:, 3:6], bg), ("specular_color", feat[:, 6:9], bg),
             ("depth", feat[:, 9:10], bg), ("normal", feat[:, 10:13], bg), ("alpha", feat[:, 13:14], zero3)]
    if debug:
        P = means3D.shape[0]
        fg = ~is_sky
        rough = torch.zeros((P, 1), device=dev)
        rough[fg] = pc.get_roughness
        metal = torch.zeros((P, 1), device=dev)
        metal[fg] = pc.get_metalness
        alb = torch.ones_like(means3D)
        alb[fg] = pc.get_albedo
        chans += [("sky_color", feat[:, 0:3] * is_sky[:, None].float(), bg), ("roughness", rough, bg),
                  ("metalness", metal, bg), ("albedo", alb, bg)]
    cols, bgs, widths = [], [], []
    for name, cval, b in chans:
        k = cval.shape[1]
        if k == 1 and not (grey or name == "alpha"):
            cval, k = cval.expand(-1, 3), 3
        cols.append(cval)
        bgs.append(b[:k])
        widths.append(k)
    nch = sum(widths)
    # without extras and with a grey background the relit rows are the features as they are
    features = feat if (not debug and grey) else torch.cat(cols, 1)
    image, radii = dgr.rasterize_channels(means3D, screenspace_points, features, opacity, scales, rotations,
                                          cov3D_precomp, torch.cat(bgs), settings, nch=nch)
    H, W = settings.image_height, settings.image_width
    imgs, c = {}, 0
    for (name, _, _), k in zip(chans, widths):
        imgs[name] = image[c:c + 1].expand(3, H, W) if k == 1 else image[c:c + 3]
        c += k
    out = {"render": imgs["render"], "viewspace_points": screenspace_points, "visibility_filter": radii > 0,
           "radii": radii}
    extras = {k: v for k, v in imgs.items() if k != "render"}
    nrm = (extras["normal"] - 0.5) * 2.
    if normal_view:
        nrm = -nrm.clone()
    extras["normal"] = nrm * sky_mask + torch.ones_like(nrm) * (1 - sky_mask)
    nref = depth_to_normal(viewpoint_camera, (extras["depth"][0] * sky_mask).unsqueeze(0)).permute(2, 0, 1)
    nref = nref * extras["alpha"].detach()
    extras["normal_ref"] = nref + torch.ones_like(nref) * (1 - sky_mask)
    out.update(extras)
    return out
