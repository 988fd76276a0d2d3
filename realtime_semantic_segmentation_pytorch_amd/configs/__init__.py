from .base_config import BaseConfig
from .my_config import MyConfig
from .parser import load_parser, get_parser

__all__ = ["BaseConfig", "MyConfig", "load_parser", "get_parser"]
