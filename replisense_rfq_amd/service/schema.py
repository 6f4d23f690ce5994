"""RFQ response schema (reference app/rfq_agent.py:20-59).

Field order defines the response JSON key order (the API returns ``.dict()``
of this model), so it is part of the byte-compatible contract.  Extra keys in
the model output are ignored, strings with thousands separators are accepted
for quantity/target_price (before-validators, rfq_agent.py:27-39).
"""
from __future__ import annotations

from typing import Optional

from pydantic import BaseModel, field_validator


class LineItem(BaseModel):
    part_number: Optional[str] = None
    description: Optional[str] = None
    quantity: Optional[int] = None
    target_price: Optional[float] = None
    currency: Optional[str] = None

    @field_validator("quantity", mode="before")
    @classmethod
    def _qty(cls, v):
        return int(v.replace(",", "")) if isinstance(v, str) else v

    @field_validator("target_price", mode="before")
    @classmethod
    def _price(cls, v):
        return float(v.replace(",", "")) if isinstance(v, str) else v


class RFQResponse(BaseModel):
    title: Optional[str] = None
    client_name: Optional[str] = None
    client_email: Optional[str] = None
    client_contact: Optional[str] = None
    client_phone: Optional[str] = None
    rfq_to: Optional[str] = None
    delivery_location: Optional[str] = None
    delivery_deadline: Optional[str] = None
    response_due_date: Optional[str] = None
    description: Optional[str] = None
    line_items: list[LineItem] = []
    requested_documents: list[str] = []
    confidence_score: float = 0.0
    missing_fields: list[str] = []
    requires_review: bool = True
    source_file: str = "email-body"
    success: bool = True
    message: str = ""

    def as_dict(self) -> dict:
        """``.dict()`` of the reference (pydantic v1 API name, same output)."""
        return self.model_dump()


FIELD_ORDER = list(RFQResponse.model_fields)
