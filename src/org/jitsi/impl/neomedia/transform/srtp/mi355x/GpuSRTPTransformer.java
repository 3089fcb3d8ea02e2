/*
 * Drop-in for SRTPTransformer (transform/srtp/SRTPTransformer.java:53-220) on
 * the MI355X engine: the same constructors and setContextFactory, and -- like
 * SRTPTransformer -- a SinglePacketTransformer, so it fits where the
 * reference holds one (DtlsPacketTransformer.java:377,549, SDesTransformEngine
 * .java:79-97).  NOT COMPILED IN THIS REPOSITORY (no JDK); see INTEGRATION.md.
 */
package org.jitsi.impl.neomedia.transform.srtp.mi355x;

public class GpuSRTPTransformer
    extends GpuTransformerBase
{
    /** SRTPTransformer(SRTPContextFactory) (:70-73) */
    public GpuSRTPTransformer(GpuSRTPContextFactory factory)
    {
        this(factory, factory);
    }

    /** SRTPTransformer(forwardFactory, reverseFactory) (:83-90) */
    public GpuSRTPTransformer(GpuSRTPContextFactory forwardFactory, GpuSRTPContextFactory reverseFactory)
    {
        super(KIND_RTP, forwardFactory, reverseFactory, null);
    }

    /** SRTPTransformer.setContextFactory (:100-125) */
    public void setContextFactory(GpuSRTPContextFactory factory, boolean forward)
    {
        replaceFactory(factory, forward);
    }
}
