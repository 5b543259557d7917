"""Drop-in mirror of the reference's ``model`` package (same module paths, class names, constructor signatures,
return tuples and state_dict keys), computed by the MI355X HIP kernels in ``arcweld``."""
