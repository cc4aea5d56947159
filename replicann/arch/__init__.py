from replicann_amd.arch import *  # noqa: F401,F403
