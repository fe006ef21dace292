from .arena import Arena, ModelLayout, ParamRef, ParamSpec  # noqa: F401
