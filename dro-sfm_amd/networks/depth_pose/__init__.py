"""Depth nets resolvable by load_class('DepthPoseNet', 'dro_sfm_amd.networks.depth_pose')."""
