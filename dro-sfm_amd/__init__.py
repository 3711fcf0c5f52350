"""dro_sfm_amd -- MI355X-native hot path of DRO-SfM (xyang9527/dro-sfm).

Drop-in replacements for the reference's recurrent depth-pose optimizer and
its self-/supervised losses.  Module paths mirror the reference package so its
class-by-name plugin loader (dro_sfm/utils/load.py:79-106) resolves them:

    dro_sfm_amd.networks.depth_pose.DepthPoseNet   (model.depth_net.name)
    dro_sfm_amd.models.SelfSupModelMF / SupModelMF (model.name)

The hot ops run as hand-written HIP kernels for gfx950 (libdro_amd.so, C ABI
in include/dro_amd.h); there is no CPU fallback.
"""
__version__ = "0.1.0"
