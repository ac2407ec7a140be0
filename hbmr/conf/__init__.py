from .configuration import Configuration  # noqa: F401
