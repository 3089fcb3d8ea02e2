/*
 * The engine-side SRTPContextFactory (transform/srtp/SRTPContextFactory.java
 * :50-68): master key, salt and the two policies become session keys on every
 * GPU.  NOT COMPILED IN THIS REPOSITORY (no JDK); see INTEGRATION.md.
 */
package org.jitsi.impl.neomedia.transform.srtp.mi355x;

import org.jitsi.impl.neomedia.transform.srtp.*;

public class GpuSRTPContextFactory
{
    final int id;

    private boolean closed;

    public GpuSRTPContextFactory(boolean sender, byte[] masterKey, byte[] masterSalt,
                                 SRTPPolicy srtpPolicy, SRTPPolicy srtcpPolicy)
    {
        id = SrtpMi355x.check(SrtpMi355x.factoryCreate(SrtpMi355x.dispatch(), sender, masterKey,
                                                        masterSalt, ints(srtpPolicy), ints(srtcpPolicy)));
    }

    private static int[] ints(SRTPPolicy p)
    {
        return new int[] { p.getEncType(), p.getEncKeyLength(), p.getAuthType(), p.getAuthKeyLength(),
                           p.getAuthTagLength(), p.getSaltKeyLength() };
    }

    /**
     * SRTPContextFactory.close() (:74-86): zeroes the keys, no new contexts.
     * Closing twice is harmless (an SRTCP transformer built from an SRTP
     * transformer shares its factories, and each closes them).
     */
    public synchronized void close()
    {
        if (!closed)
        {
            closed = true;
            SrtpMi355x.factoryClose(SrtpMi355x.dispatch(), id);
        }
    }
}
