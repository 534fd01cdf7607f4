from .launcher import init_distributed, launch, run_mapper, shutdown  # noqa: F401
from .mapper import CollectiveMapper, Context, KeyValReader  # noqa: F401
