"""Object storage for the indexing path: S3 paths, boto3-shaped clients, loopback S3 server."""
from .client import HTTPS3Client, LocalS3Client, PickleableS3ClientProxy, StreamingBody, make_client
from .errors import ClientError
from .memory import MemoryStore, parse_range
from .reader import RangedReader, open_object
from .s3path import S3Path
from .server import LoopbackS3Server

__all__ = ["ClientError", "HTTPS3Client", "LocalS3Client", "LoopbackS3Server", "MemoryStore",
           "PickleableS3ClientProxy", "RangedReader", "S3Path", "StreamingBody", "make_client", "open_object",
           "parse_range"]
