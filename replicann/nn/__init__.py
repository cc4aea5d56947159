from replicann_amd.nn import *  # noqa: F401,F403
