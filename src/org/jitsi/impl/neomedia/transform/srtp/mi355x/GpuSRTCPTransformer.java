/*
 * PacketTransformer drop-in for SRTCPTransformer (transform/srtp/
 * SRTCPTransformer.java:50-207) on the MI355X engine.  NOT COMPILED IN THIS
 * REPOSITORY (no JDK); see INTEGRATION.md.
 */
package org.jitsi.impl.neomedia.transform.srtp.mi355x;

public class GpuSRTCPTransformer
    extends GpuSRTPTransformer
{
    public GpuSRTCPTransformer(GpuSRTPContextFactory forward, GpuSRTPContextFactory reverse)
    {
        super(KIND_RTCP, forward, reverse, null);
    }

    /** SRTCPTransformer.updateFactory */
    public void updateFactory(GpuSRTPContextFactory factory, boolean forward)
    {
        setContextFactory(factory, forward);
    }
}
