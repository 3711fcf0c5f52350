"""Model classes resolvable by the reference's load_class(name, 'dro_sfm_amd.models')."""
