"""Storage errors shaped like ``botocore.exceptions.ClientError``.

The reference's control flow keys on ``error.response["Error"]["Code"]`` (``util.py:46-60`` turns a
``"404"`` from ``head_object`` into ``KeyError``; ``cloudobject.py:223-229`` creates the meta bucket on a
``"404"`` from ``head_bucket``), so the same dictionary shape is kept here.
"""
from __future__ import annotations


class ClientError(Exception):
    def __init__(self, code: str, operation_name: str, message: str = "", status: int | None = None):
        self.response = {
            "Error": {"Code": str(code), "Message": message or str(code)},
            "ResponseMetadata": {"HTTPStatusCode": int(status if status is not None else _status(code))},
        }
        self.operation_name = operation_name
        super().__init__(f"An error occurred ({code}) when calling the {operation_name} operation: {message}")


def _status(code: str) -> int:
    if str(code).isdigit():
        return int(code)
    return {"NoSuchKey": 404, "NoSuchBucket": 404, "InvalidRange": 416, "BucketAlreadyOwnedByYou": 409,
            "BucketNotEmpty": 409}.get(code, 400)


def not_found(operation_name: str, what: str = "") -> ClientError:
    return ClientError("404", operation_name, f"Not Found {what}".strip())
